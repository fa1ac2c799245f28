// ECDSA brainpoolP256r1 (SIGNATURE_TYPE 21): the EC kernels of kernels_ec.hip compiled for curve 1.
#define PZK_EC_CURVE 1
#include "kernels_ec.hip"
