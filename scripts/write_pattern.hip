// write_pattern.hip -- experiment: HBM write rate of the headline k_step's OUTPUT BYTES under
// different store orders, nothing else (no state, no logic).  4096 games x 2 envs of 16x16:
// obs [8192][256][29] float + mask [8192][256][78] int32 = 948 MB per launch, one 256-lane
// workgroup per game except the grid-stride fill.
//   mode 0  k_step's phase B: the game's obs run, then its mask run, 4 KB per workgroup iteration
//           (each wave 1 KB of it)
//   mode 1  wave-contiguous: each wave writes its own contiguous quarter of the game's obs run
//           and of its mask run
//   mode 2  wave-local cells: wave w writes the obs and mask rows of cells [64w, 64w + 64) of each
//           view (the order a barrier-free, per-wave phase A / B would produce)
//   mode 3  grid-stride fill of both buffers (torch fill_'s order; 1792 resident workgroups)
//   hipcc -O3 --offload-arch=gfx950 -o scripts/write_pattern scripts/write_pattern.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int HW = 256, P = 29, CH = 78, NV = 2;
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st(int* p, int k, int salt) {
    v4i v = {k ^ salt, k + 1, k + 2, salt};
    *reinterpret_cast<v4i*>(p) = v;
}

__global__ __launch_bounds__(256) void k_pattern(int mode, int* obs, int* mask, int G, int salt) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    if (mode == 3) {
        const long long nobs = (long long)G * NV * HW * P / 4, nmask = (long long)G * NV * HW * CH / 4;
        const long long stride = (long long)gridDim.x * 256;
        for (long long k = blockIdx.x * 256ll + t; k < nobs; k += stride) st(obs + 4 * k, (int)k, salt);
        for (long long k = blockIdx.x * 256ll + t; k < nmask; k += stride) st(mask + 4 * k, (int)k, salt);
        return;
    }
    const int g = blockIdx.x;
    int* o = obs + (size_t)g * NV * HW * P;
    int* m = mask + (size_t)g * NV * HW * CH;
    const int no = NV * HW * P / 4, nm = NV * HW * CH / 4;   // 16-B stores per game
    if (mode == 0) {
        for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
        for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
    } else if (mode == 1) {
        const int qo = no / 4, qm = nm / 4;
        for (int k = w * qo + l; k < (w + 1) * qo; k += 64) st(o + 4 * k, k, salt);
        for (int k = w * qm + l; k < (w + 1) * qm; k += 64) st(m + 4 * k, k, salt);
    } else {
        for (int v = 0; v < NV; v++) {
            const int o0 = (v * HW + 64 * w) * P / 4, on = 64 * P / 4;     // 464 stores
            const int m0 = (v * HW + 64 * w) * CH / 4, mn = 64 * CH / 4;   // 1248 stores
            for (int k = l; k < on; k += 64) st(o + 4 * (o0 + k), k, salt);
            for (int k = l; k < mn; k += 64) st(m + 4 * (m0 + k), k, salt);
        }
    }
}

int main() {
    const int G = 4096;
    int *obs, *mask;
    const size_t bo = (size_t)G * NV * HW * P * 4, bm = (size_t)G * NV * HW * CH * 4;
    hipMalloc(&obs, bo);
    hipMalloc(&mask, bm);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[4] = {"phaseB_4KB_iter", "wave_contiguous_quarter", "wave_local_cells", "grid_stride_fill"};
    for (int round = 0; round < 3; round++) {
        for (int mode = 0; mode < 4; mode++) {
            const int grid = mode == 3 ? 256 * 7 : G;
            for (int i = 0; i < 5; i++) hipLaunchKernelGGL(k_pattern, dim3(grid), dim3(256), 0, 0, mode, obs, mask, G, i);
            hipEventRecord(a);
            const int it = 50;
            for (int i = 0; i < it; i++) hipLaunchKernelGGL(k_pattern, dim3(grid), dim3(256), 0, 0, mode, obs, mask, G, i);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double us = 1000.0 * ms / it;
            printf("{\"round\": %d, \"mode\": %d, \"name\": \"%s\", \"us\": %.1f, \"TBps\": %.2f}\n", round, mode, names[mode], us,
                   (bo + bm) / us / 1e6);
        }
    }
    return hipGetLastError() != hipSuccess;
}
