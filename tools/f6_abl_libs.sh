#!/bin/bash
# Build libbert.so variants with gemm_f6.hip compiled under extra defines
# (development ablations, see gemm_f6.hip): build/abl/libbert_<name>.so
#   tools/f6_abl_libs.sh 0 64 32 ...        (-DF6_ABL=<bits>)
#   tools/f6_abl_libs.sh d12k:-DF6_DESYNC_LN=12000,-DF6_DESYNC_UP=6000 ...
# (defines naming KERN_ / I8_ also rebuild kernels.hip / gemm_i8.hip)
set -e
cd "$(dirname "$0")/.."
make -s build/libbert.so
mkdir -p build/abl
HIPFLAGS="-O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-unused-value -Wno-unused-result -fPIC -fvisibility=hidden -ffp-contract=off --offload-arch=gfx950 -Iinclude -Iembedding.cpp_amd/csrc"
OBJS="build/obj/gguf_io.o build/obj/quantize.o build/obj/quantize_model.o build/obj/synth.o build/obj/tokenizer.o build/obj/runtime.o"
for a in "$@"; do
  name=${a%%:*}
  if [[ $a == *:* ]]; then defs=${a#*:}; defs=${defs//,/ }; else defs="-DF6_ABL=$a"; fi
  /opt/rocm/bin/hipcc $HIPFLAGS $defs -c embedding.cpp_amd/csrc/gemm_f6.hip -o build/abl/gemm_f6_$name.o &
  if [[ $defs == *KERN_* ]]; then
    /opt/rocm/bin/hipcc $HIPFLAGS $defs -c embedding.cpp_amd/csrc/kernels.hip -o build/abl/kernels_$name.o &
  fi
  if [[ $defs == *I8_* ]]; then
    /opt/rocm/bin/hipcc $HIPFLAGS $defs -c embedding.cpp_amd/csrc/gemm_i8.hip -o build/abl/gemm_i8_$name.o &
  fi
done
wait
for a in "$@"; do
  name=${a%%:*}
  k=build/obj/kernels.o; [ -f build/abl/kernels_$name.o ] && k=build/abl/kernels_$name.o
  i8=build/obj/gemm_i8.o; [ -f build/abl/gemm_i8_$name.o ] && i8=build/abl/gemm_i8_$name.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o build/abl/libbert_$name.so $OBJS $k $i8 build/abl/gemm_f6_$name.o -lpthread
done
ls build/abl
