// lcv_k_fexpg.hip — kernel unit: F_fexp_glue (final-exponentiation glue steps).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_fexp_glue)
