// lcv_k_dbg.hip — kernel unit: F_dbg_fp, F_dbg_pow (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_dbg_fp)
LCV_INSTANTIATE(F_dbg_pow)
