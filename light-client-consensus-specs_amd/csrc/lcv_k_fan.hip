// lcv_k_fan.hip — kernel unit: the fan engine (latency mode) for the SOP programs F_sop_lines F_sop_acc
// F_sop_fexp F_sop_h2c and the fused Miller program F_sop_miller (lcv_sop_fan.hpp, k_sop_fan in
// lcv_functors_sop.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors_sop.hpp"

LCV_INSTANTIATE_SOP_FAN(F_sop_lines)
LCV_INSTANTIATE_SOP_FAN(F_sop_acc)
LCV_INSTANTIATE_SOP_FAN(F_sop_fexp)
LCV_INSTANTIATE_SOP_FAN(F_sop_h2c)
LCV_INSTANTIATE_SOP_FAN(F_sop_miller)
