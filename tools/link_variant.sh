#!/bin/bash
# Link a libheat.so variant in DIR from DIR/obj/*.o overrides plus build/obj/ (A/B builds: HEAT_LIB=DIR/libheat.so).
# link a libheat variant: $1 = variant dir (with obj/ overrides)
set -e
V=$1
OBJS=""
for o in capi common cpu_backend io solver topology trace transport_basic transport_loopback transport_rccl transport_tcp lds mfma stencil tb_resident tb_resident_xl0 tb_resident_xl1 tb_resident_xl2 tb_scalar tb_split tb_split_nt tb_split_rla tb_split_rlb tb_split_rlc tb_tile tb_tile_xl0 tb_tile_xl1 tb_tile_xl2; do
  if [ -f $V/obj/$o.o ]; then OBJS="$OBJS $V/obj/$o.o"; else OBJS="$OBJS build/obj/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $V/libheat.so $OBJS -fopenmp -L/opt/rocm/lib -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
