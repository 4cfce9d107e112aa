// Exhaustive device check: v_rcp_f32 plus one Newton step equals the correctly rounded 1.0F / x
// for every float x with kEpsilon <= |x| < 2^126 (both signs).  Prints the mismatch count.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/rcp_kat tools/rcp_kat.hip && tools/rcp_kat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float rcpNewton(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r, 1.0F);
    return fmaf(e, r, r);
}

__global__ void k_check(uint32_t lo, uint32_t hi, unsigned long long* bad, uint32_t* firstBad) {
    const uint64_t n = static_cast<uint64_t>(hi) - lo;
    unsigned long long local = 0;
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint32_t b = lo + static_cast<uint32_t>(i);
        for (int sgn = 0; sgn < 2; ++sgn) {
            const float x = __uint_as_float(b | (sgn ? 0x80000000u : 0u));
            const float a = 1.0F / x, f = rcpNewton(x);
            if (__float_as_uint(a) != __float_as_uint(f)) {
                ++local;
                atomicMin(firstBad, b);
            }
        }
    }
    if (local) atomicAdd(bad, local);
}

int main() {
    const float eps = 1.0e-06F, top = 0x1p126F;
    uint32_t lo, hi;
    std::memcpy(&lo, &eps, 4);
    std::memcpy(&hi, &top, 4);
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 4);
    hipMemset(bad, 0, 8);
    hipMemset(first, 0xFF, 4);
    hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, lo, hi, bad, first);
    unsigned long long h = 0;
    uint32_t f = 0;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    std::printf("checked %llu floats (both signs): %llu mismatches (first at bits 0x%08x)\n",
                2ull * (static_cast<unsigned long long>(hi) - lo), h, f);
    return h == 0 ? 0 : 1;
}
