// ECDSA brainpoolP384r1 (SIGNATURE_TYPE 25, 6 x 64-bit chunks): the EC kernels of kernels_ec.hip compiled for curve 3.
#define PZK_EC_CURVE 3
#include "kernels_ec.hip"
