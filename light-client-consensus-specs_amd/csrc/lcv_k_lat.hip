// lcv_k_lat.hip — kernel unit: the latency-mode twins F_h2c_map_lat and F_sig_lat (lcv_functors.hpp) of the SSWU
// maps and the signature decoding, built with the field products inlined (LCV_FP_CALL 0, lcv_common.hpp) and
// the square-root exponentiations in limb form, one item per wave and each chain product spread over the
// wave (LCV_POW_LF 3, lcv_field.hpp / lcv_wave.hpp).
#define LCV_KERNEL_UNIT 1
#define LCV_HD __device__
#define LCV_FP_CALL 0
#define LCV_POW_LF 3      // the sqrt chains on 28-bit limbs, each product spread over a wave (lcv_wave.hpp)
#define LCV_WAVE_ITEMS 1  // so one item per wave (lcv_launch.hpp k_wave)
#include "lcv_launch.hpp"
#include "lcv_functors.hpp"

LCV_INSTANTIATE(F_h2c_map_lat)
LCV_INSTANTIATE(F_sig_lat)
LCV_INSTANTIATE(F_dbg_pow_lat)
