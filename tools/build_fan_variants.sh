#!/bin/bash
# A/B helper: liblcv.so variants that differ only in the fan-engine unit (csrc/lcv_k_fan.hip) compiled
# with extra -D flags: VARIANTS="A: B:-DLCV_FAN_PA=1 ..." -> abp/liblcv_<name>.so (after `make`).
set -e
cd "$(dirname "$0")/../light-client-consensus-specs_amd"
mkdir -p ../abp
OBJS=$(ls build/*.o | grep -v lcv_k_fan.o)
for spec in $VARIANTS; do
  name=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-pass-failed -Ibuild $defs \
    -c csrc/lcv_k_fan.hip -o /tmp/lcv_k_fan_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../abp/liblcv_$name.so /tmp/lcv_k_fan_$name.o $OBJS \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "abp/liblcv_$name.so: $defs"
done
