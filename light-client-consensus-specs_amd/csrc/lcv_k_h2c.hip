// lcv_k_h2c.hip — kernel unit: F_h2c_map (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_h2c_map)
