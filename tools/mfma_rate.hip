// Calibration: issue rate of v_mfma_f32_16x16x4_f32 in the k_dwl accumulation pattern (8
// accumulators, 16 MFMAs per slab), one workgroup of 4 waves per CU, operands in registers or
// re-read from LDS each slab; reports shader cycles (s_memtime) and ns (s_memrealtime) per MFMA.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mfma_rate.hip -o tools/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool LDS>
__global__ __launch_bounds__(256, 1) void k_rate(float* out, unsigned long long* tm, int slabs) {
    __shared__ float sh[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) sh[i] = 0.001f * (i & 255);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    float a[2][4], b[2][4];
    for (int h = 0; h < 2; ++h)
        for (int j = 0; j < 4; ++j) { a[h][j] = 0.01f * (lane + j); b[h][j] = 0.02f * (lane - h); }
    floatx4 acc0[4], acc1[4];
    for (int s = 0; s < 4; ++s) { acc0[s] = floatx4{0.f, 0.f, 0.f, 0.f}; acc1[s] = acc0[s]; }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < slabs; ++i) {
        if constexpr (LDS) {
            const int base = ((threadIdx.x >> 6) * 1024 + (i & 3) * 256);
            for (int h = 0; h < 2; ++h)
                for (int j = 0; j < 4; ++j) { a[h][j] = sh[base + j * 32 + h * 16 + (lane & 15)]; b[h][j] = sh[base + 128 + j * 32 + h * 16 + (lane & 15)]; }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                if (j & 1) acc1[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s >> 1][j], b[s & 1][j], acc1[s], 0, 0, 0);
                else acc0[s] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s >> 1][j], b[s & 1][j], acc0[s], 0, 0, 0);
            }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float v = 0.f;
    for (int s = 0; s < 4; ++s) v += acc0[s][0] + acc1[s][1] + acc0[s][2] + acc1[s][3];
    out[blockIdx.x * 256 + threadIdx.x] = v;
    if (threadIdx.x == 0) { tm[2 * blockIdx.x] = c1 - c0; tm[2 * blockIdx.x + 1] = r1 - r0; }
}

int main() {
    float* out; unsigned long long* tm;
    CK(hipMalloc(&out, 1024 * 256 * 4)); CK(hipMalloc(&tm, 1024 * 16));
    for (int lds = 0; lds < 2; ++lds)
        for (int grid : {1, 256, 512}) {
            const int slabs = 16;
            for (int rep = 0; rep < 3; ++rep) {
                if (lds) k_rate<true><<<grid, 256>>>(out, tm, slabs);
                else k_rate<false><<<grid, 256>>>(out, tm, slabs);
            }
            CK(hipDeviceSynchronize());
            unsigned long long h[2]; CK(hipMemcpy(h, tm, 16, hipMemcpyDeviceToHost));
            const double mf = 16.0 * slabs;
            printf("lds=%d grid=%4d: %llu cycles, %.2f us for %d MFMA per wave -> %.1f cycles / MFMA, clock %.0f MHz\n",
                   lds, grid, h[0], h[1] * 0.01, (int)mf, h[0] / mf, 100.0 * h[0] / h[1]);
        }
    return 0;
}
