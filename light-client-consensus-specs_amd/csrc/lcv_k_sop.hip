// lcv_k_sop.hip — kernel unit: the SOP pairing programs F_sop_lines F_sop_acc F_sop_fexp (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors_sop.hpp"

LCV_INSTANTIATE_SOP(F_sop_lines)
LCV_INSTANTIATE_SOP(F_sop_acc)
LCV_INSTANTIATE_SOP(F_sop_fexp)
LCV_INSTANTIATE_SOP(F_sop_h2c)
