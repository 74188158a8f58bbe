// lcv_k_fexpe.hip — kernel unit: F_fexp_easy (final-exponentiation easy part).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_fexp_easy)
