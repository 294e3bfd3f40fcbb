#!/bin/bash
# Dev only (CPU side, before a GPU A/B): a copy of the product library in
# which only the fused kernel's part(s) are rebuilt with extra defines (the
# ablation switches of csrc/xm_resample_fast.hip, XM_AB_*), linked into
# xm-audio-utils_amd/<name>/libxm_audio.so.  Other objects are the product's.
#   tools/dev/ab_part.sh <name> "<defines>" [parts, default "1"]
#   e.g. tools/dev/ab_part.sh lib_nowait "-DXM_AB_NOWAIT" && tools/ab_libs.sh 2 lib lib_nowait
set -e
NAME=${1:?usage: ab_part.sh <name> "<defines>" [parts]}; DEFS=$2; PARTS=${3:-1}
cd "$(dirname "$0")/../../xm-audio-utils_amd"
make -s -j8 ARCH=gfx950 >/dev/null
OBJ=build/obj_$NAME
rm -rf $OBJ; mkdir -p $OBJ $NAME
cp -l build/obj/*.o $OBJ/
HIPFLAGS="--offload-arch=gfx950 -O3 -fvisibility=hidden -mllvm -pragma-unroll-threshold=100000000 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -Wall -Wno-unused-result -I../include -Icsrc -Ibuild/gen -fno-slp-vectorize"
# the parts in parallel (JOBS at a time, default 4)
for k in $PARTS; do rm -f $OBJ/xm_resample_fast_p$k.o; done
printf '%s\n' $PARTS | xargs -P ${JOBS:-4} -I{} /opt/rocm/bin/hipcc $HIPFLAGS $DEFS -DXM_FAST_PART={} \
  -c csrc/xm_resample_fast.hip -o $OBJ/xm_resample_fast_p{}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $NAME/libxm_audio.so $OBJ/*.o -lm -ldl -lpthread -Wl,-z,defs -Wl,--no-undefined
echo "built $NAME/libxm_audio.so ($DEFS, parts $PARTS)"
