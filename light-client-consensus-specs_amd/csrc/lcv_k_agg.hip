// lcv_k_agg.hip — kernel unit: F_agg F_agg_team F_sum F_sigroot (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_agg)
LCV_INSTANTIATE(F_agg_fold)
LCV_INSTANTIATE(F_sigroot)
LCV_INSTANTIATE_TEAM(F_agg_team)
LCV_INSTANTIATE_TEAM(F_sum)
