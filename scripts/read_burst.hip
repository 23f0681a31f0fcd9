// read_burst.hip -- experiment: the latency of a kernel's first-round reads, the pattern
// every step-kernel launch starts with (each of G workgroups loads its game's 4 KB of
// state at once).  One 256-lane workgroup per game; each lane loads 16 B of its game's
// row, the workgroup waits for them (one barrier), and lane 0 records wall_clock64()
// before and after.  Reported: the median / p90 of (data arrived - workgroup start) and
// the span of the launch, for
//   stride 4096: game g's row at g * 4 KB (the engine's cell rows; one page per game at 4 KB pages)
//   stride 0:    every game reads the same 4 KB (no page / channel spread)
//   stride 2 MB: one row per 2 MB
// each with and without a 1 GB write between launches (what the step kernel's output
// stream does to the caches and the TLBs before the next launch).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/read_burst scripts/read_burst.hip && ./scripts/read_burst
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_burst(const int4* __restrict__ src, long long stride16, unsigned long long* stamps,
                                               int* sink) {
    const unsigned long long t0 = wall_clock64();
    const int4 v = src[(long long)blockIdx.x * stride16 + threadIdx.x];
    __shared__ int acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    atomicAdd(&acc, v.x ^ v.y ^ v.z ^ v.w);
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = wall_clock64();
        if (acc == 0x7fffffff) sink[blockIdx.x] = acc;   // keeps the loads
    }
}

__global__ void k_fill(int4* p, long long n, int salt) {
    for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) p[i] = make_int4(salt, 1, 2, 3);
}

#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const int G[3] = {512, 1024, 1536};
    const long long strides[3] = {4096, 0, 2 << 20};
    const size_t src_bytes = (size_t)1536 * (2 << 20) + 4096, big = (size_t)1 << 30;
    int4 *src, *junk;
    unsigned long long* st;
    int* sink;
    CK(hipMalloc(&src, src_bytes));
    CK(hipMalloc(&junk, big));
    CK(hipMalloc(&st, 2 * 1536 * sizeof(unsigned long long)));
    CK(hipMalloc(&sink, 1536 * sizeof(int)));
    CK(hipMemset(src, 1, src_bytes));
    std::vector<unsigned long long> h(2 * 1536);
    for (int pollute = 0; pollute < 2; pollute++)
        for (long long s : strides)
            for (int g : G) {
                std::vector<double> lat, span;
                for (int rep = 0; rep < 12; rep++) {
                    if (pollute) hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, junk, (long long)(big / 16), rep);
                    hipLaunchKernelGGL(k_burst, dim3(g), dim3(256), 0, 0, src, s / 16, st, sink);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h.data(), st, 2 * g * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                    if (rep < 2) continue;
                    unsigned long long t0 = ~0ull, t1 = 0;
                    for (int b = 0; b < g; b++) {
                        t0 = std::min(t0, h[2 * b]);
                        t1 = std::max(t1, h[2 * b + 1]);
                        lat.push_back((h[2 * b + 1] - h[2 * b]) * 0.01);
                    }
                    span.push_back((t1 - t0) * 0.01);
                }
                std::sort(lat.begin(), lat.end());
                std::sort(span.begin(), span.end());
                printf("{\"pollute_1GB_write\": %d, \"stride\": %lld, \"workgroups\": %d, \"latency_us_median\": %.2f, "
                       "\"latency_us_p90\": %.2f, \"span_us_median\": %.2f}\n",
                       pollute, s, g, lat[lat.size() / 2], lat[lat.size() * 9 / 10], span[span.size() / 2]);
            }
    return 0;
}
