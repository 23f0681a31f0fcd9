// store_rate.hip -- experiment: how fast ONE workgroup (or a few) streams a game's output
// run, the bound on the step kernel's last round (the tail).  Each workgroup writes
// `bytes` contiguous bytes with 16-B stores, lanes interleaved (store k of the run on
// lane k % NT, as emit_outputs' phase B does), from registers (no LDS reads), timed with
// wall_clock64 inside the kernel.  Varies the workgroup size (64 .. 1024 lanes) and the
// number of concurrent workgroups (1, 8, 64: one per CU at most).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/store_rate scripts/store_rate.hip && ./scripts/store_rate
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

template <int NT>
__global__ __launch_bounds__(NT) void k_store(int* out, long long bytes, unsigned long long* stamps) {
    const unsigned long long t0 = wall_clock64();
    int* base = out + (long long)blockIdx.x * (bytes / 4);
    const long long n16 = bytes / 16;
    for (long long k = threadIdx.x; k < n16; k += NT) {
        v4i v = {(int)k, (int)blockIdx.x, 1, 2};
        *reinterpret_cast<v4i*>(base + 4 * k) = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = wall_clock64();
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int NT>
int run(int* out, unsigned long long* st, long long bytes, int g) {
    std::vector<unsigned long long> h(2 * g);
    std::vector<double> us;
    for (int rep = 0; rep < 10; rep++) {
        hipLaunchKernelGGL(k_store<NT>, dim3(g), dim3(NT), 0, 0, out, bytes, st);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), st, 2 * g * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        if (rep < 2) continue;
        for (int b = 0; b < g; b++) us.push_back((h[2 * b + 1] - h[2 * b]) * 0.01);
    }
    std::sort(us.begin(), us.end());
    const double med = us[us.size() / 2];
    printf("{\"lanes\": %d, \"workgroups\": %d, \"bytes_per_workgroup\": %lld, \"us_median\": %.2f, \"GBps_per_workgroup\": %.1f}\n",
           NT, g, bytes, med, bytes / (med * 1e3));
    return 0;
}

int main() {
    const long long bytes = 231424;   // one 16x16 selfplay game's obs + mask + source rows (2 envs)
    int* out;
    unsigned long long* st;
    CK(hipMalloc(&out, 64 * bytes));
    CK(hipMalloc(&st, 2 * 64 * sizeof(unsigned long long)));
    for (int g : {1, 8, 64}) {
        run<64>(out, st, bytes, g);
        run<128>(out, st, bytes, g);
        run<256>(out, st, bytes, g);
        run<512>(out, st, bytes, g);
        run<1024>(out, st, bytes, g);
    }
    return 0;
}
