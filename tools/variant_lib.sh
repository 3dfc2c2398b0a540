#!/bin/bash
# Build a variant of build/libbert.so with extra compile flags on the HIP
# sources (development A/B; run here, not on the GPU box):
#   tools/variant_lib.sh <name> "<extra hipcc flags>"  ->  build/ab/<name>/libbert.so (delete after the A/B; build/var is kept off GPU pushes)
set -e
cd "$(dirname "$0")/.."
make -s build/libbert.so
NAME=$1; FLAGS=$2
OUT=build/ab/$NAME
mkdir -p "$OUT"
HIPFLAGS="-O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form -Wno-unused-value -Wno-unused-result -fPIC -fvisibility=hidden -ffp-contract=off --offload-arch=gfx950 -Iinclude -Iembedding.cpp_amd/csrc"
for f in kernels gemm_i8; do
  /opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c embedding.cpp_amd/csrc/$f.hip -o "$OUT/$f.o" &
done
wait
HOST=$(ls build/obj/*.o | grep -v -E '/(kernels|gemm_i8)\.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT/libbert.so" $HOST "$OUT/kernels.o" "$OUT/gemm_i8.o" -lpthread
cp build/BUILD_INFO "$OUT/BUILD_INFO" 2>/dev/null || true
# a variant is not the clean HEAD build: say which one it is
printf ' variant=%s (%s)' "$NAME" "$FLAGS" >> "$OUT/BUILD_INFO"
echo "$OUT/libbert.so ($FLAGS)"
