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
//   mode 4  as 3 with one constant value in every store (what a fill writes)
//   mode 5  as 3 with non-temporal stores
//   mode 6  as 0 (phase B order) with one constant value in every store
//   mode 7  hipMemsetD32Async of both buffers (the runtime's fill: 256 workgroups of 256 lanes)
//   mode 8  as 3 on 256 workgroups (one per CU), mode 9 on 512, mode 10 on 1024
//   mode 11 as 0 (phase B order, 4096 workgroups) with only waves 0-1 storing (128 lanes)
//   mode 12 as 0 with only wave 0 storing (64 lanes)
//   mode 13 as 8 (256 workgroups) with non-temporal stores
//   mode 14 games' runs (phase B order) by 256 persistent workgroups (game b, b + 256, ...)
//   mode 15 games' runs by 1024 persistent workgroups, mode 16 by 512
//   mode 17 as 0 with each game's runs started at a rotated 4 KB chunk (g mod 8), wrapping round
//   mode 18 as 0 with the obs and mask runs interleaved chunk by chunk
//   mode 19 as 0 with 32 contiguous bytes per lane (two adjacent 16-B stores, 8 KB per iteration)
//   mode 20 as 0 with each run written back to front
//   mode 21 as 0 with every workgroup writing the mask run first, then the obs run
//   mode 22 as 0 with a permuted game order (odd games g and g ^ 2 swapped)
//   mode 23 games' runs by 256 persistent workgroups, each a contiguous block of G / 256 games
//   mode 24 as 23 on 512 workgroups, mode 25 on 1024, mode 26 on 128
//   mode 27 block fill: each of 256 workgroups writes its contiguous 1/256 of each buffer
//   mode 28 emit proxy: as 8 (grid-stride, 256 workgroups), every 16-B store's words built from
//           the game state (int4 per cell, 4 KB per game): obs stores read their cell(s), mask
//           stores their cell and its 4 neighbours -- the emit kernel of a logic / emit split
//   mode 29 as 28 on 512 workgroups, mode 30 on 1792
//   mode 31 pipelined emit proxy (timing only): 256 workgroups walk the grid-stride window of 4 KB
//           chunks; each step's game state (4 KB, one int4 per lane) is loaded D = 8 steps ahead
//           into registers, parked in LDS when its step comes, and the chunk's words are built from
//           LDS (cell + 4 neighbours) -- what a logic / emit split's emit kernel would have to do
//   mode 32 as 31 with D = 16, mode 33 as 31 on 512 workgroups
//   mode 34 wave-private emit proxy: each wave walks the window in 1 KB chunks; lane L loads the
//           state of cell c0 - 16 + L (the chunk's cells and their row neighbours, one int4 per
//           lane) D = 16 chunks ahead in a statically unrolled ring (no register rotation, no
//           barrier); the words are built with cross-lane reads.  Mode 35: D = 24, mode 36: D = 8
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
__device__ __forceinline__ void stc(int* p, int salt) {
    v4i v = {salt, salt, salt, salt};
    *reinterpret_cast<v4i*>(p) = v;
}
__device__ __forceinline__ void stnt(int* p, int k, int salt) {
    v4i v = {k ^ salt, k + 1, k + 2, salt};
    __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(p));
}

__device__ __forceinline__ int cellword(const int4* __restrict__ state, int g, int c) {
    const int4 u = state[(size_t)g * HW + c];
    return (u.x & 15) | ((u.x >> 4 & 3) << 4) | ((u.z & 7) << 8) | (u.w & 0xff) << 12;
}

// one buffer of the proxy: store k (16 B) of game g's run; constant divisors, 32-bit math
template <int WIDTH, bool NB>
__device__ __forceinline__ void emit_direct(int* out, const int4* __restrict__ state, int G, int salt) {
    constexpr int PER = NV * HW * WIDTH / 4;   // 16-B stores per game
    const unsigned n = (unsigned)G * PER, stride = gridDim.x * 256u;
    for (unsigned k = blockIdx.x * 256u + threadIdx.x; k < n; k += stride) {
        const unsigned g = k / PER, w0 = 4 * (k - g * PER), c2 = w0 / WIDTH, ch = w0 - c2 * WIDTH, c = c2 & (HW - 1);
        const int x = c & 15, y = c >> 4;
        int acc = cellword(state, g, c);
        if (NB) {
            if (y > 0) acc ^= cellword(state, g, c - 16) << 1;
            if (x < 15) acc ^= cellword(state, g, c + 1) << 2;
            if (y < 15) acc ^= cellword(state, g, c + 16) << 3;
            if (x > 0) acc ^= cellword(state, g, c - 1) << 4;
        } else if (ch + 3 >= WIDTH && c + 1 < HW) {
            acc ^= cellword(state, g, c + 1) << 5;
        }
        v4i v;
        for (int q = 0; q < 4; q++) v[q] = ((acc >> ((ch + q) & 31)) & 1) ^ salt;
        *reinterpret_cast<v4i*>(out + 4 * (size_t)k) = v;
    }
}

__global__ __launch_bounds__(256) void k_emit_proxy(int* obs, int* mask, const int4* __restrict__ state, int G, int salt) {
    emit_direct<P, false>(obs, state, G, salt);
    emit_direct<CH, true>(mask, state, G, salt);
}

template <int D, int WIDTH, bool NB>
__device__ __forceinline__ void emit_pipe(int* out, const int4* __restrict__ state, int G, int salt, int* lw) {
    constexpr int PER = NV * HW * WIDTH / 4;
    const int t = threadIdx.x;
    const unsigned n = (unsigned)G * PER, stride = gridDim.x * 256u, first = blockIdx.x * 256u;
    int4 ring[D];
#pragma unroll
    for (int d = 0; d < D; d++) ring[d] = state[(size_t)min((unsigned)G - 1, (first + d * stride) / PER) * HW + t];
    for (unsigned k0 = first; k0 < n; k0 += stride) {
        const int4 u = ring[0];
#pragma unroll
        for (int d = 0; d + 1 < D; d++) ring[d] = ring[d + 1];
        ring[D - 1] = state[(size_t)min((unsigned)G - 1, (k0 + D * stride) / PER) * HW + t];
        __syncthreads();
        lw[t] = (u.x & 15) | ((u.x >> 4 & 3) << 4) | ((u.z & 7) << 8) | (u.w & 0xff) << 12;
        __syncthreads();
        const unsigned k = k0 + t;
        if (k < n) {
            const unsigned g0 = k0 / PER, w0 = 4 * (k - g0 * PER), c2 = w0 / WIDTH, ch = w0 - c2 * WIDTH, c = c2 & (HW - 1);
            const int x = c & 15, y = c >> 4;
            int acc = lw[c];
            if (NB) {
                if (y > 0) acc ^= lw[c - 16] << 1;
                if (x < 15) acc ^= lw[c + 1] << 2;
                if (y < 15) acc ^= lw[c + 16] << 3;
                if (x > 0) acc ^= lw[c - 1] << 4;
            }
            v4i v;
            for (int q = 0; q < 4; q++) v[q] = ((acc >> ((ch + q) & 31)) & 1) ^ salt;
            *reinterpret_cast<v4i*>(out + 4 * (size_t)k) = v;
        }
    }
}

template <int D>
__global__ __launch_bounds__(256) void k_emit_pipe(int* obs, int* mask, const int4* __restrict__ state, int G, int salt) {
    __shared__ int lw[HW];   // the step's game, one word per cell
    emit_pipe<D, P, false>(obs, state, G, salt, lw);
    emit_pipe<D, CH, true>(mask, state, G, salt, lw);
}

template <int D, int WIDTH, bool NB>
__device__ __forceinline__ void emit_wave(int* out, const int4* __restrict__ state, int G, int salt) {
    constexpr int PER = NV * HW * WIDTH / 4;   // 16-B stores per game
    const int lane = threadIdx.x & 63;
    const unsigned nw = gridDim.x * 4u, gw = blockIdx.x * 4u + (threadIdx.x >> 6);
    const unsigned nch = ((unsigned)G * PER + 63) / 64;   // 1 KB chunks
    auto cell_of = [&](unsigned j, unsigned& g, int& c0) {   // chunk j: its game and first cell
        const unsigned k0 = j * 64u;
        g = min(k0 / PER, (unsigned)G - 1);
        c0 = (int)((4 * (k0 - g * PER) / WIDTH) & (HW - 1));
    };
    auto load = [&](unsigned j) {
        unsigned g;
        int c0;
        cell_of(min(j, nch - 1), g, c0);
        return state[(size_t)g * HW + min(max(c0 - 16 + lane, 0), HW - 1)];
    };
    int4 ring[D];
#pragma unroll
    for (int d = 0; d < D; d++) ring[d] = load(gw + d * nw);
    for (unsigned j0 = gw; j0 < nch; j0 += D * nw) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const unsigned j = min(j0 + d * nw, nch - 1);   // past the end: rewrites the last chunk (same words)
            const int4 u = ring[d];
            ring[d] = load(j0 + d * nw + D * nw);
            {
                unsigned g;
                int c0;
                cell_of(j, g, c0);
                const int word = (u.x & 15) | ((u.x >> 4 & 3) << 4) | ((u.z & 7) << 8) | (u.w & 0xff) << 12;
                const unsigned k = j * 64u + lane, w0 = 4 * (k - g * PER), c2 = w0 / WIDTH, ch = w0 - c2 * WIDTH;
                const int c = (int)(c2 & (HW - 1)), rel = min(max(c - c0 + 16, 0), 63);
                int acc = __shfl(word, rel);
                if (NB) {
                    acc ^= __shfl(word, max(rel - 16, 0)) << 1;
                    acc ^= __shfl(word, min(rel + 1, 63)) << 2;
                    acc ^= __shfl(word, min(rel + 16, 63)) << 3;
                    acc ^= __shfl(word, max(rel - 1, 0)) << 4;
                }
                v4i v;
                for (int q = 0; q < 4; q++) v[q] = ((acc >> ((ch + q) & 31)) & 1) ^ salt;
                if (k < (unsigned)G * PER) *reinterpret_cast<v4i*>(out + 4 * (size_t)k) = v;
            }
        }
    }
}
template <int D>
__global__ __launch_bounds__(256) void k_emit_wave(int* obs, int* mask, const int4* __restrict__ state, int G, int salt) {
    emit_wave<D, P, false>(obs, state, G, salt);
    emit_wave<D, CH, true>(mask, state, G, salt);
}

__global__ __launch_bounds__(256) void k_pattern(int mode, int* obs, int* mask, int G, int salt) {
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    if (mode >= 8 && mode <= 10) mode = 3;
    if (mode == 13) mode = 5;
    if (mode >= 23 && mode <= 26) {   // block-distributed games: workgroup b writes games [b * G / n, (b + 1) * G / n)
        const int no = NV * HW * P / 4, nm = NV * HW * CH / 4, per = G / gridDim.x;
        for (int g = blockIdx.x * per; g < (blockIdx.x + 1) * per; g++) {
            int* o = obs + (size_t)g * NV * HW * P;
            int* m = mask + (size_t)g * NV * HW * CH;
            for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
            for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
        }
        return;
    }
    if (mode == 27) {
        const long long nobs = (long long)G * NV * HW * P / 4, nmask = (long long)G * NV * HW * CH / 4;
        const long long po = nobs / gridDim.x, pm = nmask / gridDim.x;
        for (long long k = blockIdx.x * po + t; k < (blockIdx.x + 1) * po; k += 256) st(obs + 4 * k, (int)k, salt);
        for (long long k = blockIdx.x * pm + t; k < (blockIdx.x + 1) * pm; k += 256) st(mask + 4 * k, (int)k, salt);
        return;
    }
    if (mode >= 14 && mode <= 16) {
        const int no = NV * HW * P / 4, nm = NV * HW * CH / 4;
        for (int g = blockIdx.x; g < G; g += gridDim.x) {
            int* o = obs + (size_t)g * NV * HW * P;
            int* m = mask + (size_t)g * NV * HW * CH;
            for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
            for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
        }
        return;
    }
    if (mode == 3 || mode == 4 || mode == 5) {
        const long long nobs = (long long)G * NV * HW * P / 4, nmask = (long long)G * NV * HW * CH / 4;
        const long long stride = (long long)gridDim.x * 256;
        for (long long k = blockIdx.x * 256ll + t; k < nobs; k += stride)
            mode == 3 ? st(obs + 4 * k, (int)k, salt) : mode == 4 ? stc(obs + 4 * k, salt) : stnt(obs + 4 * k, (int)k, salt);
        for (long long k = blockIdx.x * 256ll + t; k < nmask; k += stride)
            mode == 3 ? st(mask + 4 * k, (int)k, salt) : mode == 4 ? stc(mask + 4 * k, salt) : stnt(mask + 4 * k, (int)k, salt);
        return;
    }
    const int g = blockIdx.x;
    if (mode == 22) {   // swizzle: which game a workgroup writes (a permutation of 0..G-1)
        const int gg = (g & 1) ? (g ^ 2) : g;
        int* o = obs + (size_t)gg * NV * HW * P;
        int* m = mask + (size_t)gg * NV * HW * CH;
        const int no = NV * HW * P / 4, nm = NV * HW * CH / 4;
        for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
        for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
        return;
    }
    int* o = obs + (size_t)g * NV * HW * P;
    int* m = mask + (size_t)g * NV * HW * CH;
    const int no = NV * HW * P / 4, nm = NV * HW * CH / 4;   // 16-B stores per game
    if (mode == 0) {
        for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
        for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
    } else if (mode == 17) {
        const int rot = (g & 7) * 256;   // in 16-B stores: 4 KB chunks
        for (int k = t; k < no; k += 256) { const int j = (k + rot) % no; st(o + 4 * j, j, salt); }
        for (int k = t; k < nm; k += 256) { const int j = (k + rot) % nm; st(m + 4 * j, j, salt); }
    } else if (mode == 18) {
        for (int k = t; k < nm; k += 256) {
            if (k < no) st(o + 4 * k, k, salt);
            st(m + 4 * k, k, salt);
        }
    } else if (mode == 19) {
        for (int k = 2 * t; k < no; k += 512) { st(o + 4 * k, k, salt); if (k + 1 < no) st(o + 4 * k + 4, k + 1, salt); }
        for (int k = 2 * t; k < nm; k += 512) { st(m + 4 * k, k, salt); if (k + 1 < nm) st(m + 4 * k + 4, k + 1, salt); }
    } else if (mode == 20) {
        for (int k = t; k < no; k += 256) { const int j = no - 1 - k; st(o + 4 * j, j, salt); }
        for (int k = t; k < nm; k += 256) { const int j = nm - 1 - k; st(m + 4 * j, j, salt); }
    } else if (mode == 21) {
        for (int k = t; k < nm; k += 256) st(m + 4 * k, k, salt);
        for (int k = t; k < no; k += 256) st(o + 4 * k, k, salt);
    } else if (mode == 11 || mode == 12) {
        const int nt = mode == 11 ? 128 : 64;
        if (t >= nt) return;
        for (int k = t; k < no; k += nt) st(o + 4 * k, k, salt);
        for (int k = t; k < nm; k += nt) st(m + 4 * k, k, salt);
    } else if (mode == 6) {
        for (int k = t; k < no; k += 256) stc(o + 4 * k, salt);
        for (int k = t; k < nm; k += 256) stc(m + 4 * k, salt);
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
    int* state;   // 4 KB of int4 cells per game, arbitrary contents
    hipMalloc(&state, (size_t)G * HW * 16);
    hipMemset(state, 0x5a, (size_t)G * HW * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[37] = {"phaseB_4KB_iter", "wave_contiguous_quarter", "wave_local_cells", "grid_stride_fill",
                             "grid_stride_constant", "grid_stride_nontemporal", "phaseB_constant", "hipMemsetD32",
                             "grid_stride_256wg", "grid_stride_512wg", "grid_stride_1024wg", "phaseB_2waves", "phaseB_1wave",
                             "grid_stride_256wg_nt", "games_256_persistent", "games_1024_persistent", "games_512_persistent",
                             "phaseB_rotated_start", "phaseB_obs_mask_interleaved", "phaseB_32B_per_lane", "phaseB_back_to_front",
                             "phaseB_mask_first", "phaseB_game_swizzle", "games_256_block", "games_512_block",
                             "games_1024_block", "games_128_block", "block_fill_256wg", "emit_proxy_256wg",
                             "emit_proxy_512wg", "emit_proxy_1792wg", "emit_pipe_D8_256wg",
                             "emit_pipe_D16_256wg", "emit_pipe_D8_512wg", "emit_wave_D16_256wg",
                             "emit_wave_D24_256wg", "emit_wave_D8_256wg"};
    auto launch = [&](int mode, int grid, int i) {
        if (mode >= 34) {
            if (mode == 34) hipLaunchKernelGGL(k_emit_wave<16>, dim3(256), dim3(256), 0, 0, obs, mask, (const int4*)state, G, i);
            if (mode == 35) hipLaunchKernelGGL(k_emit_wave<24>, dim3(256), dim3(256), 0, 0, obs, mask, (const int4*)state, G, i);
            if (mode == 36) hipLaunchKernelGGL(k_emit_wave<8>, dim3(256), dim3(256), 0, 0, obs, mask, (const int4*)state, G, i);
        } else if (mode >= 31) {
            if (mode == 32)
                hipLaunchKernelGGL(k_emit_pipe<16>, dim3(256), dim3(256), 0, 0, obs, mask, (const int4*)state, G, i);
            else
                hipLaunchKernelGGL(k_emit_pipe<8>, dim3(mode == 33 ? 512 : 256), dim3(256), 0, 0, obs, mask, (const int4*)state, G, i);
        } else if (mode >= 28) {
            hipLaunchKernelGGL(k_emit_proxy, dim3(mode == 28 ? 256 : mode == 29 ? 512 : 1792), dim3(256), 0, 0, obs, mask,
                               (const int4*)state, G, i);
        } else if (mode == 7) {
            hipMemsetD32Async((hipDeviceptr_t)obs, i, bo / 4, 0);
            hipMemsetD32Async((hipDeviceptr_t)mask, i, bm / 4, 0);
        } else {
            hipLaunchKernelGGL(k_pattern, dim3(grid), dim3(256), 0, 0, mode, obs, mask, G, i);
        }
    };
    for (int round = 0; round < 3; round++) {
        for (int mode = 0; mode < 37; mode++) {
            const int grid = (mode >= 3 && mode <= 5) ? 256 * 7 : (mode == 8 || mode == 13 || mode == 14 || mode == 23 || mode == 27) ? 256
                           : (mode == 9 || mode == 16 || mode == 24) ? 512 : (mode == 10 || mode == 15 || mode == 25) ? 1024
                           : mode == 26 ? 128 : G;
            for (int i = 0; i < 5; i++) launch(mode, grid, i);
            hipEventRecord(a);
            const int it = 50;
            for (int i = 0; i < it; i++) launch(mode, grid, i);
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
