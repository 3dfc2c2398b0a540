// exp_probe.hip — can soft_max's exp lookup (ggml's fp16 table, entry
// 0x8000 | m = fp16(expf(-h(m))) built with the host's libm) be computed in
// registers?  For every m the kernels can look up (fp16 magnitudes below the
// table's constant run, and the run itself up to +inf), compare device candidates against the host table and
// count the mismatches (development probe; prints one JSON line).
//   hipcc --offload-arch=gfx950 -O2 -Iembedding.cpp_amd/csrc tools/exp_probe.hip -o build/exp_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#include "ggml_formats.h"

using namespace bertamd;

__device__ __forceinline__ uint16_t dev_f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
__device__ __forceinline__ float dev_h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

// candidates: 0 __expf (v_exp_f32 of x * log2 e), 1 expf (ocml), 2 exp2f(x * log2e) with
// the product split (x * log2e in two parts), 3 (float) exp((double) x)
__global__ void probe(int n, uint16_t *out) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n) return;
    const float x = -dev_h2f((uint16_t)m);
    out[0 * n + m] = dev_f2h(__expf(x));
    out[1 * n + m] = dev_f2h(expf(x));
    const float hi = x * 1.4426950216293335f, lo = __builtin_fmaf(x, 1.4426950216293335f, -hi) + x * 1.9259629911783487e-08f;
    out[2 * n + m] = dev_f2h(__builtin_amdgcn_exp2f(hi) * __builtin_amdgcn_exp2f(lo));
    out[3 * n + m] = dev_f2h((float)exp((double)x));
}

int main() {
    std::vector<uint16_t> tab(65536);
    for (int i = 0; i < 65536; i++) tab[i] = f32_to_f16(expf(f16_to_f32((uint16_t)i)));
    const uint16_t cst = tab[0xfbff];
    int n = 0x7c00;
    while (n > 0 && tab[0x8000 | (n - 1)] == cst) n--;
    constexpr int NC = 4;
    const int neg_n = n;
    n = 0x7c01;  // every magnitude up to +inf (masked keys): the constant-0 run too
    uint16_t *d;
    if (hipMalloc(&d, (size_t)NC * n * 2) != hipSuccess) return 1;
    probe<<<(n + 255) / 256, 256>>>(n, d);
    std::vector<uint16_t> h((size_t)NC * n);
    if (hipMemcpy(h.data(), d, h.size() * 2, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::printf("{\"neg_n\": %d, \"checked\": %d", neg_n, n);
    for (int c = 0; c < NC; c++) {
        int bad = 0, first = -1;
        for (int m = 0; m < n; m++)
            if (h[(size_t)c * n + m] != tab[0x8000 | m]) {
                if (first < 0) first = m;
                bad++;
            }
        std::printf(", \"cand%d_mismatch\": %d, \"cand%d_first\": %d", c, bad, c, first);
    }
    std::printf("}\n");
    (void)hipFree(d);
    return 0;
}
