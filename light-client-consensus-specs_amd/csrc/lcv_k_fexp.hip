// lcv_k_fexp.hip — kernel unit: F_fexp_pow (exponentiation by |x| in the cyclotomic subgroup; see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_fexp_pow)
