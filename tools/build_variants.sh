#!/bin/bash
# A/B helper: liblcv.so variants that differ only in one unit (UNIT, default the fan engine's
# csrc/lcv_k_fan.hip; lcv_hip for the driver) compiled with extra -D flags:
# VARIANTS="A: B:-DLCV_FAN_SPLIT=0 ..." -> abp/liblcv_<name>.so (after `make`).
set -e
cd "$(dirname "$0")/../light-client-consensus-specs_amd"
mkdir -p ../abp
UNIT=${UNIT:-lcv_k_fan}
OBJS=$(ls build/*.o | grep -v "$UNIT.o")
for spec in $VARIANTS; do
  name=${spec%%:*}; defs=${spec#*:}; defs=${defs//,/ }
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-pass-failed -Ibuild $defs \
    -c csrc/$UNIT.hip -o /tmp/${UNIT}_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../abp/liblcv_$name.so /tmp/${UNIT}_$name.o $OBJS \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "abp/liblcv_$name.so: $defs"
done
