// lcv_k_ssz.hip — kernel unit: F_nsc_team F_pre F_merkle F_htr_sc F_msg_import F_msg_import_b0 F_verdict F_export_g2 F_export_g1 F_export_fp12 F_import_pq (see lcv_launch.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE_TEAM(F_nsc_team)
LCV_INSTANTIATE(F_pre)
LCV_INSTANTIATE(F_merkle)
LCV_INSTANTIATE(F_htr_sc)
LCV_INSTANTIATE(F_msg_import)
LCV_INSTANTIATE(F_msg_import_b0)
LCV_INSTANTIATE(F_verdict)
LCV_INSTANTIATE(F_export_g2)
LCV_INSTANTIATE(F_export_g1)
LCV_INSTANTIATE(F_export_fp12)
LCV_INSTANTIATE(F_import_pq)
