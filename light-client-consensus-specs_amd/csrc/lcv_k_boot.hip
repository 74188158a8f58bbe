// lcv_k_boot.hip — kernel unit: F_bootstrap (initialize_light_client_store checks; see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_bootstrap)
