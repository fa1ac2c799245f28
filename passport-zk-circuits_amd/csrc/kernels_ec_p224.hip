// ECDSA secp224r1 (SIGNATURE_TYPE 24, 7 x 32-bit chunks): the EC kernels of kernels_ec.hip compiled for curve 2.
#define PZK_EC_CURVE 2
#include "kernels_ec.hip"
