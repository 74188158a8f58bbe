// lcv_k_engine.hip — kernel unit: F_eng_miller F_eng_fexp F_eng_h2c F_eng_g2sub (team interpreter of the generated pairing
// programs, lcv_engine.hpp).  The interpreter's one Fp multiplication is inlined (LCV_FP_CALL 0).
#define LCV_FP_CALL 0
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors_eng.hpp"

LCV_INSTANTIATE_TEAM(F_eng_miller)
LCV_INSTANTIATE_TEAM(F_eng_fexp)
LCV_INSTANTIATE_TEAM(F_eng_h2c)
LCV_INSTANTIATE_TEAM(F_eng_g2sub)
