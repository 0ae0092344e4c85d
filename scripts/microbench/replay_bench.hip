// The lazy out-table catch-up (k_rows_adam<false, true>: p-only g = 0 replays) in isolation:
// R rows of d = 128 with geometric lags (mean ~4.7 steps, C3's 64-walk batch), replayed by
//   0: the scaled sequences (sqrtf, IEEE division; Markstein for / bc2s)   [r04e]
//   1: dw::replay_g0 (the box forms; the box header in the history's row 0)
//   2: the box forms one step at a time, no checks
//   3: one wave per row, 2 elements per lane (more loads in flight per wave)
//   4: one wave per two rows
//   5: as 3 with a 2048-block grid
//   6: no replay (the row loads and the p store alone: the traffic's floor)
//   7-8: the traffic alone with dwordx2 / dwordx4 loads (a row per wave / two)
//   9-11: mode 1 software-pipelined (the next row's loads before this row's replay), grids
//         of 16384 / 4096 / 65536 blocks
// Prints the mean kernel time per variant and checks every variant gives variant 0's bits.
//   hipcc -O3 --offload-arch=gfx950 -I include scripts/microbench/replay_bench.hip \
//         -o scripts/microbench/replay_bench
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../deepwalk-and-node2vec_amd/csrc/dw_common.h"

template <int MODE>
__global__ void __launch_bounds__(512)
    k_replay(float *__restrict__ p, const float *__restrict__ m, const float *__restrict__ v,
             const int32_t *__restrict__ last, int32_t d, const uint32_t *__restrict__ rows,
             int64_t n, const float *__restrict__ hist, int32_t upto) {
    const int e = threadIdx.x;
    const bool live = e < d;
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t r = rows[i];
        const int32_t from = __builtin_amdgcn_readfirstlane(last[r]);
        const int64_t o = r * d + e;
        float pr[1] = {live ? p[o] : 0.f}, mr[1] = {live ? m[o] : 0.f};
        float vr[1] = {live ? v[o] : 0.f};
        if (MODE == 0) {
            for (int32_t s = from + 1; s <= upto; ++s) {
                const dw::AdamScalars h = dw::hist_at(hist, s);
                if (h.wd == 0.f) {
                    dw::adam_elem_g0(pr[0], mr[0], vr[0], h);
                } else {
                    float z = 0.f;
                    dw::adam_elem(pr[0], z, mr[0], vr[0], h);
                }
            }
        } else if (MODE == 1) {
            dw::replay_g0(pr, mr, vr, hist, from, upto, dw::hist_box_from(hist));
        } else if (MODE == 6) {   // no replay: the loads and the store alone
            pr[0] = pr[0] + mr[0] * vr[0] * static_cast<float>(upto - from) * 0.f;
        } else {
            const dw::const_float *hc = (const dw::const_float *)hist;
            for (int32_t s = from + 1; s <= upto; ++s)
                dw::adam_elem_g0_box(pr[0], mr[0], vr[0], dw::hist_at_const(hc + 8 * s));
        }
        if (live) p[o] = pr[0];
    }
}


// One wave per row (RPW rows per wave, their loads in flight together), VPL elements per lane
// (element lane + 64 k): the replay through dw::replay_g0.
template <int VPL, int RPW>
__global__ void __launch_bounds__(256)
    k_replay_wave(float *__restrict__ p, const float *__restrict__ m, const float *__restrict__ v,
                  const int32_t *__restrict__ last, int32_t d, const uint32_t *__restrict__ rows,
                  int64_t n, const float *__restrict__ hist, int32_t upto) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW;
    const int64_t wstride = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6) * RPW;
    for (int64_t i0 = w0; i0 < n; i0 += wstride) {
        float pr[RPW][VPL], mr[RPW][VPL], vr[RPW][VPL];
        int64_t rr[RPW];
        int32_t fr[RPW];
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            const bool ok = i0 + j < n;
            rr[j] = ok ? static_cast<int64_t>(rows[i0 + j]) : 0;
            fr[j] = ok ? __builtin_amdgcn_readfirstlane(last[rr[j]]) : upto;
#pragma unroll
            for (int k = 0; k < VPL; ++k) {
                const int e = lane + 64 * k;
                const bool live = ok && e < d && fr[j] < upto;
                const int64_t o = rr[j] * d + e;
                pr[j][k] = live ? p[o] : 0.f;
                mr[j][k] = live ? m[o] : 0.f;
                vr[j][k] = live ? v[o] : 0.f;
            }
        }
#pragma unroll
        for (int j = 0; j < RPW; ++j) {
            dw::replay_g0(pr[j], mr[j], vr[j], hist, fr[j], upto, dw::hist_box_from(hist));
#pragma unroll
            for (int k = 0; k < VPL; ++k) {
                const int e = lane + 64 * k;
                if (i0 + j < n && e < d && fr[j] < upto) p[rr[j] * d + e] = pr[j][k];
            }
        }
    }
}

// The traffic alone with wider loads: each lane loads VEC floats of a row (dword / dwordx2 /
// dwordx4), 128 / VEC lanes per row, 64 / (128 / VEC) rows per wave.
template <int VEC>
__global__ void __launch_bounds__(256)
    k_traffic(float *__restrict__ p, const float *__restrict__ m, const float *__restrict__ v,
              const int32_t *__restrict__ last, const uint32_t *__restrict__ rows, int64_t n,
              int32_t upto) {
    typedef float __attribute__((ext_vector_type(VEC))) fv;
    constexpr int LPR = 128 / VEC;            // lanes per row
    constexpr int RPW = 64 / LPR;             // rows per wave
    const int lane = threadIdx.x & 63;
    const int64_t w = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int64_t i = w * RPW + lane / LPR;
    if (i >= n) return;
    const int64_t r = rows[i];
    const int32_t from = last[r];
    const int64_t o = r * 128 + (lane % LPR) * VEC;
    fv pp = *reinterpret_cast<const fv *>(p + o);
    const fv mm = *reinterpret_cast<const fv *>(m + o);
    const fv vv = *reinterpret_cast<const fv *>(v + o);
    pp = pp + mm * vv * static_cast<float>(upto - from) * 0.f;
    *reinterpret_cast<fv *>(p + o) = pp;
}

// k_replay<1> with the next row's loads issued before the current row's replay (software
// pipelined: a wave's loads stay in flight while it computes).
__global__ void __launch_bounds__(512)
    k_replay_pf(float *__restrict__ p, const float *__restrict__ m, const float *__restrict__ v,
                const int32_t *__restrict__ last, int32_t d, const uint32_t *__restrict__ rows,
                int64_t n, const float *__restrict__ hist, int32_t upto) {
    const int e = threadIdx.x;
    const bool live = e < d;
    const int32_t box_from = dw::hist_box_from(hist);
    int64_t i = blockIdx.x;
    if (i >= n) return;
    int64_t r = rows[i];
    int32_t from = __builtin_amdgcn_readfirstlane(last[r]);
    float pn = live ? p[r * d + e] : 0.f, mn = live ? m[r * d + e] : 0.f;
    float vn = live ? v[r * d + e] : 0.f;
    for (; i < n; i += gridDim.x) {
        float pr[1] = {pn}, mr[1] = {mn}, vr[1] = {vn};
        const int64_t rc = r;
        const int32_t fc = from;
        const int64_t j = i + gridDim.x;
        if (j < n) {   // the next row's loads, in flight during this row's replay
            r = rows[j];
            from = __builtin_amdgcn_readfirstlane(last[r]);
            pn = live ? p[r * d + e] : 0.f;
            mn = live ? m[r * d + e] : 0.f;
            vn = live ? v[r * d + e] : 0.f;
        }
        dw::replay_g0(pr, mr, vr, hist, fc, upto, box_from);
        if (live) p[rc * d + e] = pr[0];
    }
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static double urand() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (rng_state >> 11) * 0x1p-53;
}

int main(int argc, char **argv) {
    const int64_t R = argc > 1 ? atoll(argv[1]) : 224000, V = 1 << 20;
    const int d = 128, T = 400, reps = argc > 2 ? atoi(argv[2]) : 20;
    std::vector<float> hp(V * d), hm(V * d), hv(V * d), hist(8 * (T + 1));
    std::vector<int32_t> hlast(V);
    std::vector<uint32_t> hrows(R);
    for (int64_t i = 0; i < V * d; ++i) {
        hp[i] = (float)(urand() - 0.5) * 0.01f;
        hm[i] = (float)((urand() - 0.5) * 2e-8);
        hv[i] = (float)(urand() * 1e-17);
    }
    for (int64_t r = 0; r < V; ++r) {
        int lag = 1;
        while (urand() > 0.21 && lag < 200) ++lag;   // geometric, mean ~4.7
        hlast[r] = T - lag;
    }
    for (int64_t i = 0; i < R; ++i) hrows[i] = (uint32_t)((i * 2654435761ull) % V);
    for (int s = 0; s <= T; ++s) {   // sharding.hist_row: lr .01, betas (.9, .999), eps 1e-8
        const int t = s < 1 ? 1 : s;
        const double bc1 = 1.0 - pow(0.9, t), bc2 = 1.0 - pow(0.999, t);
        float *h = &hist[8 * s];
        h[0] = 0.1f;
        h[1] = 0.999f;
        h[2] = (float)(1.0 - 0.999);
        h[3] = (float)sqrt(bc2);
        h[4] = (float)(-0.01 / bc1);
        h[5] = 1e-8f;
        h[6] = 0.f;
        volatile float one = 1.f;
        h[7] = one / h[3];
    }
    {   // the box header (every step's scalars are in the box)
        const uint32_t tag = DW_HIST_BOX_TAG, from1 = 1;
        memcpy(&hist[0], &tag, 4);
        memcpy(&hist[1], &from1, 4);
    }
    float *dp, *dm, *dv, *dh, *dp0;
    int32_t *dl;
    uint32_t *dr;
    hipMalloc(&dp, V * d * 4);
    hipMalloc(&dp0, V * d * 4);
    hipMalloc(&dm, V * d * 4);
    hipMalloc(&dv, V * d * 4);
    hipMalloc(&dh, hist.size() * 4);
    hipMalloc(&dl, V * 4);
    hipMalloc(&dr, R * 4);
    hipMemcpy(dp0, hp.data(), V * d * 4, hipMemcpyHostToDevice);
    hipMemcpy(dm, hm.data(), V * d * 4, hipMemcpyHostToDevice);
    hipMemcpy(dv, hv.data(), V * d * 4, hipMemcpyHostToDevice);
    hipMemcpy(dh, hist.data(), hist.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dl, hlast.data(), V * 4, hipMemcpyHostToDevice);
    hipMemcpy(dr, hrows.data(), R * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> out[12];
    const unsigned grid = R < 65536 ? (unsigned)R : 65536u;
    for (int mode = 0; mode < 12; ++mode) {
        float tot = 0.f;
        for (int k = 0; k < reps + 2; ++k) {
            hipMemcpy(dp, dp0, V * d * 4, hipMemcpyDeviceToDevice);
            hipEventRecord(a, 0);
            if (mode == 0)
                hipLaunchKernelGGL(k_replay<0>, dim3(grid), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 1)
                hipLaunchKernelGGL(k_replay<1>, dim3(grid), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 2)
                hipLaunchKernelGGL(k_replay<2>, dim3(grid), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 3)   // wave per row, 2 elements per lane
                hipLaunchKernelGGL((k_replay_wave<2, 1>), dim3((R + 3) / 4), dim3(256), 0, 0, dp,
                                   dm, dv, dl, d, dr, R, dh, T - 1);
            else if (mode == 4)   // two rows per wave
                hipLaunchKernelGGL((k_replay_wave<2, 2>), dim3((R + 7) / 8), dim3(256), 0, 0, dp,
                                   dm, dv, dl, d, dr, R, dh, T - 1);
            else if (mode == 5)   // wave per row, capped grid (grid-stride)
                hipLaunchKernelGGL((k_replay_wave<2, 1>), dim3(2048), dim3(256), 0, 0, dp, dm, dv,
                                   dl, d, dr, R, dh, T - 1);
            else if (mode == 6)   // the memory traffic alone
                hipLaunchKernelGGL(k_replay<6>, dim3(grid), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 7)   // dwordx2, a row per wave
                hipLaunchKernelGGL(k_traffic<2>, dim3((R + 3) / 4), dim3(256), 0, 0, dp, dm, dv,
                                   dl, dr, R, T - 1);
            else if (mode == 9)   // pipelined, 16384 blocks
                hipLaunchKernelGGL(k_replay_pf, dim3(16384), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 10)  // pipelined, 4096 blocks
                hipLaunchKernelGGL(k_replay_pf, dim3(4096), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else if (mode == 11)  // pipelined, 65536 blocks
                hipLaunchKernelGGL(k_replay_pf, dim3(grid), dim3(d), 0, 0, dp, dm, dv, dl, d, dr,
                                   R, dh, T - 1);
            else                  // dwordx4, two rows per wave
                hipLaunchKernelGGL(k_traffic<4>, dim3((R / 2 + 3) / 4), dim3(256), 0, 0, dp, dm,
                                   dv, dl, dr, R, T - 1);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (k >= 2) tot += ms;
        }
        out[mode].resize(V * d);
        hipMemcpy(out[mode].data(), dp, V * d * 4, hipMemcpyDeviceToHost);
        printf("mode %d: %.1f us per launch (%lld rows)\n", mode, 1e3 * tot / reps, (long long)R);
    }
    bool all = true;
    for (int mode : {1, 2, 3, 4, 5, 9, 10, 11}) {
        const bool same = memcmp(out[0].data(), out[mode].data(), V * d * 4) == 0;
        printf("mode %d == mode 0 bits: %s\n", mode, same ? "yes" : "NO");
        all = all && same;
    }
    return all ? 0 : 1;
}
