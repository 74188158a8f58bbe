// lcv_k_signer.hip — kernel unit: F_sk_to_pk F_sign (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_sk_to_pk)
LCV_INSTANTIATE(F_sign)
