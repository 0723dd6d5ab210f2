// Calibration of rocprofv3 FETCH_SIZE on gfx950 for the access shapes libsacx uses (the
// MICROARCH guide calibrates only 16-B-per-lane streaming reads, which FETCH_SIZE tallies at
// half their bytes).  Each kernel reads a fresh 64 MiB buffer exactly once (every line misses
// L2 once) in one shape; run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and divide the
// reported FETCH_SIZE (KB) by 65,536 KB:
//   k_v4    16 B per lane, a wave-instruction = 1 KiB contiguous   (global_load_dwordx4)
//   k_dw    4 B per lane, a wave-instruction = 256 B contiguous     (global_load_dword)
//   k_frag  4 B per lane in k_gemm's MFMA operand shape: 16 lanes x 4 B = 64 B of a row, 4 rows
//           per instruction; the other 64 B of each 128-B line by another workgroup
// build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_v4(const float4* __restrict__ a, float* out, size_t n4) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) { float4 v = a[i]; s += v.x + v.y + v.z + v.w; }
    if (s == 12345.f) out[0] = s;
}
__global__ void k_dw(const float* __restrict__ a, float* out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == 12345.f) out[0] = s;
}
// rows of 256 floats (1 KiB); workgroup b takes column half (b & 1) -- 16 columns of each
// 32-column block -- of a band of rows; lane (r, grp) of wave w reads row 16 j + 4 grp + w,
// column 32 c + 16 half + r
__global__ void k_frag(const float* __restrict__ a, float* out, int rows) {
    const int half = blockIdx.x & 1, band = blockIdx.x >> 1;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, grp = lane >> 4;
    float s = 0.f;
    for (int j = 0; j < 4; ++j) {
        const int row = band * 64 + 16 * j + 4 * grp + w;
        if (row >= rows) break;
        for (int c = 0; c < 8; ++c) s += a[(size_t)row * 256 + 32 * c + 16 * half + r];
    }
    if (s == 12345.f) out[0] = s;
}

int main() {
    const size_t bytes = 64u << 20, n = bytes / 4;
    float *a, *b, *c, *out;
    CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&c, bytes)); CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes)); CK(hipMemset(c, 0, bytes));
    // push the buffers out of L2 and the 256 MiB Infinity Cache before each read
    float* flush; CK(hipMalloc(&flush, 512u << 20));
    auto evict = [&]() { (void)hipMemset(flush, 1, 512u << 20); (void)hipDeviceSynchronize(); };
    evict(); k_v4<<<2048, 256>>>((const float4*)a, out, n / 4); CK(hipDeviceSynchronize());
    evict(); k_dw<<<2048, 256>>>(b, out, n); CK(hipDeviceSynchronize());
    evict(); k_frag<<<2 * (int)(n / 256 / 64), 256>>>(c, out, (int)(n / 256)); CK(hipDeviceSynchronize());
    printf("each kernel read %zu KB once\n", bytes >> 10);
    return 0;
}
