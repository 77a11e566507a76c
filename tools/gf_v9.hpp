// gf_v9.hpp — single-barrier, role-split fused guided-filter kernel for radii 1..4 on
// quad-aligned geometry.
//
// Same arithmetic as gf3d_fused_kernel (gf_fused.hpp; reference guided_filter.rs:117-164): stage 1
// (u = box_r(v)) in exact f64 window sums, stage 2 (box_r(a), box_r(b)) in f32, a z-march per
// 64 x 32 output tile with the stage-2 z-window in a register ring. What changes is the schedule:
//
//   * The x-window sums of BOTH stages run across lanes (DPP wave shifts of 4-element quads), so
//     the only LDS hand-offs left are the two y-window inputs: Hx (stage-1 x-sums, f64) and Hab
//     (stage-2 x-sums of (a, b)). Both are double-buffered by slice parity, as is the output tile.
//   * With every hand-off double-buffered, one iteration runs, for four different slices,
//         A  P12(i+1)  z-window (running f64) and x-sums of v            -> Hx[(i+1)&1]
//         B  P3(i)     y-sums of Hx -> u -> a, b -> x-sums of (a, b)      -> Hab[i&1]
//         C  P5(i-1)   y-sums of Hab -> ring -> z-window -> out(i-1-R)    -> Lout[(i-1)&1]
//         D  store     Lout[i&1] -> out(i-2-R)
//     with ONE barrier per iteration (gf_fused.hpp needs two). tools/trace_steps showed the
//     two-barrier march spending a large part of each interval with a SIMD's youngest wave
//     running its last phase alone.
//   * Roles: waves 0..NW3-1 run B, the other waves run A (two passes of E2 rows each); every
//     wave runs C and, for the first 512 threads, D. The two roles are separate loops, so the
//     compiler allocates registers for the larger role, not for both: the stage-2 ring (40 VGPRs)
//     plus either the stage-1 running sums and their prefetch, or the pointwise prefetch.
//   * v for the pointwise stage and for the output is loaded straight into registers one step
//     ahead (no staging through LDS).
//
// Lanes: A owns E2 quads (3 rows of <= 20 quads per wave), B owns (quad, K3 rows) of the E1 apron
// (3 row groups of 18 quads per wave), C owns (column, 2 rows) of the tile. Requirements (checked
// by the host, v9_eligible): x0, nx, onx and the row/slice pitches multiples of 4 and 4-element
// aligned bases, so every quad is wholly inside or outside the domain / output box and
// out-of-domain quads read 0 through kBadOff. Clamped-window counts are computed per position off
// the interior fast path.
#pragma once

#include <cstdlib>

#include "gf_fused_variants.hpp"

#ifndef GF_V9_K3
#define GF_V9_K3 2
#endif
#ifndef GF_V9_STORE_AUX
#define GF_V9_STORE_AUX 2  // output store cache policy (2 = nt, 16 = sc1: drop the line from L2)
#endif

namespace zt {

template <int R>
struct V9Config {
    static constexpr int NT = 1024, NWAVE = NT / 64;
    static constexpr int TX = 64, TY = 32, W = 2 * R + 1, W3 = W * W * W;
    static constexpr int E2Y = TY + 4 * R, E1Y = TY + 2 * R;
    // role B (P3): quads x in [x0 - 4, x0 + 68) (covers E1 for R <= 4), K3 rows per lane
    static constexpr int Q3X = 18, HXC = 4 * Q3X;
    static constexpr int K3 = GF_V9_K3;
    static constexpr int NRP = E1Y / K3;                // row groups
    static constexpr int RP3 = 64 / Q3X;                // row groups per wave (3)
    static constexpr int NW3 = (NRP + RP3 - 1) / RP3;   // role-B waves
    // role A (P12): E2 quads start NB2 quads left of x0
    static constexpr int NW12 = NWAVE - NW3;            // role-A waves
    static constexpr int NB2 = (2 * R + 3) / 4;
    static constexpr int Q2X = 16 + 2 * NB2;            // quads per E2 row
    static constexpr int RPW = 64 / Q2X;                // E2 rows per wave and pass
    static constexpr int NQP1 = (E2Y + RPW * NW12 - 1) / (RPW * NW12);  // passes
    // Hx: two planes (elements 0-1 and 2-3 of every quad) of [E2Y rows][PQ] double2. With
    // K3 * PQ * 16 = 32 mod 256 the 18-quad row groups of a role-B wave (K3 rows apart) fall on
    // disjoint banks in every ds_read_b128 lane group.
    static constexpr int PQ = K3 == 2 ? 25 : 26;
    static constexpr int p2m4(int x) { return x + ((2 - x % 4) + 4) % 4; }
    static constexpr int PB = p2m4(TX);                 // Hab row pitch (float2)
    static constexpr int K5 = TX * TY / NT;             // outputs per thread (2)
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_HXP = al(E2Y * PQ * 16);    // one plane
    static constexpr int SZ_HX = 2 * SZ_HXP, SZ_HAB = al(E1Y * PB * 8);
    static constexpr int SZ_OUT = al(TY * TX * 4), SZ_RCP = al((W3 + 1) * 4);
    static constexpr int OFF_HX = 0, OFF_HAB = OFF_HX + 2 * SZ_HX;
    static constexpr int OFF_OUT = OFF_HAB + 2 * SZ_HAB, OFF_RCP = OFF_OUT + 2 * SZ_OUT;
    static constexpr int LDS_BYTES = OFF_RCP + SZ_RCP;
    static_assert(R >= 1 && R <= 4, "v9 handles radii 1..4");
    static_assert(E1Y % K3 == 0 && RPW >= 1 && NW3 < NWAVE && K5 == 2, "layout");
    static_assert(K3 == 2, "P3 shares one core between exactly two rows");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// x-window sums of W = 2R+1 along a row held as one quad per lane (lanes = consecutive quads).
// in[e] is this lane's element e; the neighbours' partial sums arrive by DPP wave shifts (lane
// l-1 holds the left quad, l+1 the right one). out[e] = sum of the row over [4q+e-R, 4q+e+R].
// Lanes whose neighbour is not their row's quad (row ends inside a wave) produce values the
// caller drops.
template <int R, typename T, typename Shift>
__device__ __forceinline__ void quad_xsums(const T (&in)[4], T (&out)[4], Shift&& shift) {
    // suffix sums S[k] = in[k..3] go right, prefix sums P[k] = in[0..k] go left
    T S[4], P[4];
    S[3] = in[3];
    S[2] = in[2] + S[3];
    S[1] = in[1] + S[2];
    S[0] = in[0] + S[1];
    P[0] = in[0];
    P[1] = P[0] + in[1];
    P[2] = P[1] + in[2];
    P[3] = S[0];
    T SL[4], PR[4];  // left neighbour's S, right neighbour's P (only the indices used)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= 4 - R) SL[k] = shift(S[k], true);   // left part of e: SL[e + 4 - R], e < R
        if (k <= R - 1) PR[k] = shift(P[k], false);  // right part of e: PR[e + R - 4], e >= 4 - R
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        // own part: in[max(0, e-R) .. min(3, e+R)]
        const int lo = e - R < 0 ? 0 : e - R, hi = e + R > 3 ? 3 : e + R;
        T own;
        if (lo == 0 && hi == 3) own = S[0];
        else if (lo == 0) own = P[hi];
        else if (hi == 3) own = S[lo];
        else {
            own = in[lo];
            for (int j = lo + 1; j <= hi; ++j) own = own + in[j];
        }
        T acc = own;
        if (e - R < 0) acc = SL[e + 4 - R] + acc;
        if (e + R > 3) acc = acc + PR[e + R - 4];
        out[e] = acc;
    }
}

__device__ __forceinline__ float dpp_f32(float v, bool from_lower) {
    const int x = __float_as_int(v);
    return __int_as_float(from_lower ? __builtin_amdgcn_update_dpp(0, x, 0x138, 0xF, 0xF, false)
                                     : __builtin_amdgcn_update_dpp(0, x, 0x130, 0xF, 0xF, false));
}

template <int R, typename TIn, typename TOut>
__global__ __launch_bounds__(1024) void gf3d_v9_kernel(GFParams p) {
    using C = V9Config<R>;
    constexpr int TX = C::TX, TY = C::TY, W = C::W, K5 = C::K5;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* rcp_tab = reinterpret_cast<float*>(smem + C::OFF_RCP);
    // correctly rounded reciprocals of every window count (Markstein needs RN(1/c) exactly);
    // published by the prologue barrier
    for (int c = threadIdx.x; c <= C::W3; c += C::NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;

    // ---- tile (XCD-aware, as gf3d_fused_kernel) --------------------------------------------
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int gtx = p.tiles_x, gty = p.tiles_y, ntiles = gtx * gty;
    const int seg = lid / ntiles;
    int t = lid % ntiles, tile_x, tile_y;
    {
        const int stx = 8, sty = 4;
        const int full_y = gty / sty * sty, per_srow = gtx * sty;
        if (t < full_y * gtx) {
            const int sr = t / per_srow, r = t % per_srow;
            const int full_x = gtx / stx * stx;
            if (r < full_x * sty) {
                tile_x = (r / (stx * sty)) * stx + r % stx;
                tile_y = sr * sty + (r / stx) % sty;
            } else {
                const int rr = r - full_x * sty, w = gtx - full_x;
                tile_x = full_x + rr % w;
                tile_y = sr * sty + rr / w;
            }
        } else {
            t -= full_y * gtx;
            tile_x = t % gtx;
            tile_y = full_y + t / gtx;
        }
    }
    const int x0 = p.ox0 + tile_x * TX, y0 = p.oy0 + tile_y * TY;
    const int ox_end = p.ox0 + p.onx, oy_end = p.oy0 + p.ony;
    const int zo_begin = p.oz0 + seg * p.zseg;
    const int zo_end = min(zo_begin + p.zseg, p.oz0 + p.onz);
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const float eps = p.eps;
    const uint32_t slice_bytes = (uint32_t)((int64_t)(p.ny - 1) * p.in_sy + p.nx) * ESZ;
    const uint32_t oslice_bytes = (uint32_t)((int64_t)(p.ony - 1) * p.out_sy + p.onx) * OSZ;
    const int sy = (int)p.in_sy, osy = (int)p.out_sy;
    const char* in_base = static_cast<const char*>(p.in);
    const char* out_base = static_cast<const char*>(p.out);
    const int zlo = p.zlo, zspan = p.zhi - p.zlo;
    const int64_t sstride = p.in_sz * ESZ, osstride = p.out_sz * OSZ;
    // descriptor of input slice z (num_records 0 outside the planes present: reads give 0)
    auto rs_at = [&](int z) -> rsrc_t {
        const bool ok = (unsigned)(z - zlo) < (unsigned)zspan;
        return make_rsrc(in_base + (ok ? (int64_t)(z - p.in_z0) * sstride : 0),
                         ok ? slice_bytes : 0u);
    };
    const int zc_begin = zo_begin - R, zc_end = zo_end + R;
    const bool xy_interior = x0 - 2 * R >= 0 && x0 + TX + 2 * R <= nx && y0 - 2 * R >= 0 &&
                             y0 + TY + 2 * R <= ny;
    constexpr float kW3 = (float)C::W3;
    const float rcp_w3 = p.rcp_w3;
    // the wave index as a provably uniform value: the role branch below is a scalar branch
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64);
    // Per-lane geometry (offsets, counts) is derived from `tid` where it is used instead of once
    // before the march: `tid` passes through an empty asm at the top of every step, so the
    // compiler cannot hoist those loop-invariant values and keep them live across the loop,
    // where they spilled (and every scratch reload waits with vmcnt(0) for all prefetches).
    int tid = threadIdx.x;

    char* const Hx0 = smem + C::OFF_HX;
    float2* const Hab0 = reinterpret_cast<float2*>(smem + C::OFF_HAB);
    float* const Lout0 = reinterpret_cast<float*>(smem + C::OFF_OUT);
    // Hx plane h of parity par: [E2Y][PQ] double2
    auto Hx = [&](int par, int h) {
        return reinterpret_cast<double2*>(Hx0 + par * C::SZ_HX + h * C::SZ_HXP);
    };
    auto Hab = [&](int par) { return Hab0 + par * (C::SZ_HAB / 8); };
    auto Lout = [&](int par) { return Lout0 + par * (C::SZ_OUT / 4); };

    // ==== C: (column, 2 rows) of the tile on every wave ========================================
    float v5[K5];  // v of the output slice (prefetched a step ahead)
    auto load_v5 = [&](int z) {
        const int col5 = tid % TX, seg5 = tid / TX;
        const int ox5 = x0 + col5, oy5 = y0 + seg5 * K5;
        const rsrc_t r = rs_at(z);
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = oy5 + j;
            const int off = (ox5 < ox_end && oy < oy_end) ? (oy * sy + ox5) * ESZ : kBadOff;
            v5[j] = Buf<TIn>::load(r, off);
        }
    };
    f2 ring[W][K5], pre[K5];  // stage-2 z-window: prefix/suffix blocks of W (see gf_fused.hpp)
#pragma unroll
    for (int s = 0; s < W; ++s)
#pragma unroll
        for (int j = 0; j < K5; ++j) ring[s][j] = (f2){0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < K5; ++j) pre[j] = (f2){0.0f, 0.0f};
    // y-window of Hab -> slice sums -> ring; out(zc - R) = v*mean(a) + mean(b) -> Lout
    auto do_p5 = [&](int zc, const float2* hab, float* lout, auto slot_c) {
        const int col5 = tid % TX, seg5 = tid / TX;
        const int ox5 = x0 + col5, oy5 = y0 + seg5 * K5;
        const f2* src = reinterpret_cast<const f2*>(hab) + (seg5 * K5) * C::PB + col5;
        f2 vin[K5 + 2 * R], s2[K5];
#pragma unroll
        for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = src[j * C::PB];
        core_window_sums<R, K5>(vin, s2);
        constexpr int P = decltype(slot_c)::value;
        f2 AB[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            pre[j] = (P == 0) ? s2[j] : pre[j] + s2[j];
            if constexpr (P == W - 1) AB[j] = pre[j];
            else AB[j] = ring[(P + 1) % W][j] + pre[j];
            ring[P][j] = s2[j];
        }
        if constexpr (P == W - 1) {
#pragma unroll
            for (int q = W - 2; q >= 0; --q)
#pragma unroll
                for (int j = 0; j < K5; ++j) ring[q][j] = ring[q][j] + ring[q + 1][j];
        }
        const int zo = zc - R;
        const bool interior = xy_interior && zo - R >= 0 && zo + R < nz;
        const float cz = (float)clamped_count(zo, nz, R);
        f2 fc[K5], rc[K5], q[K5], r[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            if (interior) {
                fc[j] = (f2){kW3, kW3};
                rc[j] = (f2){rcp_w3, rcp_w3};
            } else {
                // (positions outside the domain can give counts outside [0, W^3]: clamp the index)
                const float c = fminf(fmaxf((float)(clamped_count(ox5, nx, R) *
                                                    clamped_count(oy5 + j, ny, R)) * cz, 0.0f),
                                      kW3);
                const float rr = rcp_tab[(int)c];
                fc[j] = (f2){c, c};
                rc[j] = (f2){rr, rr};
            }
        }
        // (sum as f32) / (count as f32) for a and b together (exact: Markstein)
#pragma unroll
        for (int j = 0; j < K5; ++j) q[j] = AB[j] * rc[j];
#pragma unroll
        for (int j = 0; j < K5; ++j) r[j] = pk_fma(-q[j], fc[j], AB[j]);
#pragma unroll
        for (int j = 0; j < K5; ++j) q[j] = pk_fma(r[j], rc[j], q[j]);
#pragma unroll
        for (int j = 0; j < K5; ++j)  // v *= mean(a); v += mean(b): two roundings (:144-162)
            lout[(seg5 * K5 + j) * TX + col5] = __fadd_rn(__fmul_rn(v5[j], q[j].x), q[j].y);
    };

    // ==== D: Lout -> global, one 16-byte quad per thread (threads 0..511) ======================
    auto store_out = [&](const float* lout, int zs) {
        const unsigned nzo = (unsigned)(zo_end - zo_begin);
        const rsrc_t ro = make_rsrc(out_base + (int64_t)(zs - p.oz0) * osstride,
                                    (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u);
        const bool act = tid < TX / 4 * TY;
        const int row = act ? tid / (TX / 4) : 0, cq = act ? tid % (TX / 4) : 0;
        const float4 o4 = *reinterpret_cast<const float4*>(lout + row * TX + 4 * cq);
        const float o[4] = {o4.x, o4.y, o4.z, o4.w};
        const int ox = x0 + 4 * cq, oy = y0 + row;
        const bool in = act && ox < ox_end && oy < oy_end;
        const int off = in ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
        if constexpr (std::is_same<TOut, float>::value && GF_V9_STORE_AUX != 2) {
            const u32x4 qv = {__float_as_uint(o[0]), __float_as_uint(o[1]),
                              __float_as_uint(o[2]), __float_as_uint(o[3])};
            __builtin_amdgcn_raw_buffer_store_b128(qv, ro, off, 0, GF_V9_STORE_AUX);
        } else {
            Quad<TOut>::store(o, ro, off);
        }
    };

    // The march: iteration i runs D (out(i-2-R)), the role's phase, C (P5(i-1)) and one
    // barrier. It is unrolled by W so P5's ring slot (slice i-1's position in its block of W)
    // is a compile-time constant: a runtime slot, even dispatched by a scalar switch, makes the
    // compiler shuffle the ring between registers at the merge and spill it. The step count
    // is rounded up to whole blocks; steps past the last output emit nothing (their stores
    // carry an empty descriptor, their loads read outside the slab as 0).
    const int n_blocks = (zc_end - zc_begin + 2 + W - 1) / W;
    auto march = [&](auto&& pre_step, auto&& role_step) {
        int i = zc_begin;
        for (int blk = 0; blk < n_blocks; ++blk) {
            static_for<0, W>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                __asm__ volatile("" : "+v"(tid));
                const int par = i & 1;
                pre_step(i);
                store_out(Lout(par), i - 2 - R);
                role_step(i, par);
                if (i > zc_begin)
                    do_p5(i - 1, Hab(par ^ 1), Lout(par ^ 1),
                          std::integral_constant<int, (k + W - 1) % W>{});
                load_v5(i - R);
                lds_barrier();
                ++i;
            });
        }
    };

    if (wave < C::NW3) {
        // ==== role B: P3 on (quad, K3 rows) of the E1 apron ===================================
        constexpr int K3 = C::K3;
        struct Geo3 {
            int rp, q3, gx3, gy3;
            bool p3_lane, x3in, p3_out;
        };
        auto geo3 = [&]() {
            Geo3 g;
            const int lane = tid % 64;
            const int rp_raw = wave * C::RP3 + lane / C::Q3X;
            g.q3 = lane % C::Q3X;
            g.rp = rp_raw < C::NRP ? rp_raw : C::NRP - 1;  // idle lanes read a valid row
            g.p3_lane = lane < C::RP3 * C::Q3X && rp_raw < C::NRP;
            g.gx3 = x0 - 4 + 4 * g.q3;          // x of element 0
            g.gy3 = y0 - R + K3 * g.rp;         // y of the first row
            g.x3in = g.gx3 >= 0 && g.gx3 < nx;  // quad wholly in or out
            g.p3_out = g.p3_lane && g.q3 >= 1 && g.q3 <= 16;  // writes Hab cols 4(q3-1)..+3
            return g;
        };
        float v3[K3][4];  // v of the P3 slice (prefetched a step ahead)
        auto load_v3 = [&](int zc) {
            const Geo3 g = geo3();
            const int gx3 = g.gx3, gy3 = g.gy3;
            const bool p3_lane = g.p3_lane, x3in = g.x3in;
            const rsrc_t r = rs_at(zc);
#pragma unroll
            for (int rr = 0; rr < K3; ++rr) {
                const int gy = gy3 + rr;
                const int off =
                    (p3_lane && x3in && gy >= 0 && gy < ny) ? (gy * sy + gx3) * ESZ : kBadOff;
                Quad<TIn>::load(r, off, v3[rr]);
            }
        };
        // U = y-window sum (f64, exact) of Hx -> u -> a, b for each of the K3 rows, then the
        // x-sums of (a, b) across lanes -> Hab. The 2R rows common to the K3 windows (the core)
        // are summed once per plane; each row then adds its edge row, runs the pointwise stage
        // and its x-sums and leaves for Hab before the next row starts (one row's (a, b) live at
        // a time: the stage-2 ring keeps its registers).
        auto do_p3 = [&](int zc, int par, float2* hab) {
            const Geo3 g = geo3();
            const int rp = g.rp, q3 = g.q3, gx3 = g.gx3, gy3 = g.gy3;
            const bool x3in = g.x3in, p3_out = g.p3_out;
            const bool zin = zc >= 0 && zc < nz;
            const bool fast = xy_interior && zc - R >= 0 && zc + R < nz;  // count = W^3
            const float cz = (float)clamped_count(zc, nz, R);
            const double2* src[2] = {Hx(par, 0) + (K3 * rp) * C::PQ + q3,
                                     Hx(par, 1) + (K3 * rp) * C::PQ + q3};
            double2 core[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                // rows 1..2R in two halves with scheduling fences: at most R+1 rows in flight
                core[h] = src[h][C::PQ];
#pragma unroll
                for (int j = 2; j <= R; ++j) {
                    const double2 t2 = src[h][j * C::PQ];
                    core[h].x = core[h].x + t2.x;
                    core[h].y = core[h].y + t2.y;
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = R + 1; j <= 2 * R; ++j) {
                    const double2 t2 = src[h][j * C::PQ];
                    core[h].x = core[h].x + t2.x;
                    core[h].y = core[h].y + t2.y;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int r = 0; r < K3; ++r) {
                const bool ok = fast || (zin && x3in && gy3 + r >= 0 && gy3 + r < ny);
                const float cyz = (float)clamped_count(gy3 + r, ny, R) * cz;
                f2 ab[4];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // row r's window = rows r .. r+2R = the core + edge row 0 or 2R+1
                    const double2 edge = src[h][(r == 0 ? 0 : 2 * R + 1) * C::PQ];
                    const f2 Uf = (f2){(float)(edge.x + core[h].x), (float)(edge.y + core[h].y)};
                    const int e0 = 2 * h, e1 = 2 * h + 1;
                    const f2 vv = (f2){v3[r][e0], v3[r][e1]};
                    f2 fc, rc;
                    if (fast) {
                        fc = (f2){kW3, kW3};
                        rc = (f2){rcp_w3, rcp_w3};
                    } else {
                        // (counts outside [0, W^3] off the domain: clamp the table index)
                        const float c0 = fminf(
                            fmaxf((float)clamped_count(gx3 + e0, nx, R) * cyz, 0.f), kW3);
                        const float c1 = fminf(
                            fmaxf((float)clamped_count(gx3 + e1, nx, R) * cyz, 0.f), kW3);
                        fc = (f2){c0, c1};
                        rc = (f2){rcp_tab[(int)c0], rcp_tab[(int)c1]};
                    }
                    // u = RN(U / c) (Markstein with rcp = RN(1/c)); s = (v-u)^2;
                    // a = s/(s+eps); b = (1-a)*u  (guided_filter.rs:126-137)
                    f2 q = Uf * rc;
                    f2 rr = pk_fma(-q, fc, Uf);
                    const f2 u = pk_fma(rr, rc, q);
                    f2 sq = vv - u;
                    sq = sq * sq;
                    const f2 den = sq + (f2){eps, eps};
                    f2 y = (f2){__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
                    const f2 e = pk_fma(-den, y, (f2){1.0f, 1.0f});
                    y = pk_fma(e, y, y);
                    q = sq * y;
                    rr = pk_fma(-den, q, sq);
                    const f2 a = pk_fma(rr, y, q);
                    const f2 bb = ((f2){1.0f, 1.0f} - a) * u;
                    // zero outside the domain: the clamped window sums of stage 2 (the interior
                    // fast path is inside the domain by construction)
                    ab[e0] = ok ? (f2){a.x, bb.x} : (f2){0.f, 0.f};
                    ab[e1] = ok ? (f2){a.y, bb.y} : (f2){0.f, 0.f};
                    __builtin_amdgcn_sched_barrier(0);
                }
                // x-sums of a, then of b (one f32 quad's prefix/suffix temporaries at a time)
                const float av[4] = {ab[0].x, ab[1].x, ab[2].x, ab[3].x};
                const float bv[4] = {ab[0].y, ab[1].y, ab[2].y, ab[3].y};
                auto shift = [](float v, bool lower) { return dpp_f32(v, lower); };
                float xa[4], xb[4];
                quad_xsums<R>(av, xa, shift);
                __builtin_amdgcn_sched_barrier(0);
                quad_xsums<R>(bv, xb, shift);
                if (p3_out) {
                    float4* dst =
                        reinterpret_cast<float4*>(hab + (K3 * rp + r) * C::PB + 4 * (q3 - 1));
                    dst[0] = make_float4(xa[0], xb[0], xa[1], xb[1]);
                    dst[1] = make_float4(xa[2], xb[2], xa[3], xb[3]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        // prologue: role A writes Hx of slice zc_begin; prefetch step zc_begin
        load_v3(zc_begin);
        load_v5(zc_begin - 1 - R);
        lds_barrier();
        march([](int) {},
              [&](int i, int par) {
                  do_p3(i, par, Hab(par));
                  load_v3(i + 1);
              });
    } else {
        // ==== role A: P12 on E2 quads, NQP1 passes per wave ====================================
        const int wa = wave - C::NW3;
        auto p12_geo = [&](int k, int& off, int& row, int& qi, bool& ok) {
            const int lane = tid % 64;
            row = (k * C::NW12 + wa) * C::RPW + lane / C::Q2X;
            const int q = lane % C::Q2X;
            const bool valid = lane < C::RPW * C::Q2X && row < C::E2Y;
            const int gx = x0 - 4 * C::NB2 + 4 * q, gy = y0 - 2 * R + row;
            const bool in = valid && gy >= 0 && gy < ny && gx >= 0 && gx < nx;
            off = in ? (gy * sy + gx) * ESZ : kBadOff;
            qi = q - C::NB2 + 1;  // Hx quad column (x0 - 4 origin)
            ok = valid && qi >= 0 && qi < C::Q3X;
        };
        auto q1off = [&](int k) {
            int off, row, qi;
            bool ok;
            p12_geo(k, off, row, qi, ok);
            return off;
        };
        // running z-window of v: seed with slices [zc_begin-1-R, zc_begin-1+R] clamped to the
        // domain; every step adds the entering and subtracts the leaving slice (both read 0
        // outside the planes present), so the window stays exact
        double zv[C::NQP1][4];
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) zv[k][e] = 0.0;
        {
            const int za = max(zc_begin - 1 - R, 0), zb_ = min(zc_begin - 1 + R, nz - 1);
            for (int z = za; z <= zb_; ++z) {
                const rsrc_t rs = rs_at(z);
#pragma unroll
                for (int k = 0; k < C::NQP1; ++k) {
                    float v[4];
                    Quad<TIn>::load(rs, q1off(k), v);
#pragma unroll
                    for (int e = 0; e < 4; ++e) zv[k][e] += (double)v[e];
                }
            }
        }
        float pa[C::NQP1][4], ps[C::NQP1][4];
        // stage-1 slice zc: the entering slice zc+R is prefetched a step ahead; the leaving slice
        // zc-R-1 (read 2R+1 steps earlier, an L2/MALL hit) only at the top of its step, so its
        // registers are not live across P5
        auto load_pa = [&](int zc) {
            const rsrc_t ra = rs_at(zc + R);
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) Quad<TIn>::load(ra, q1off(k), pa[k]);
        };
        auto load_ps = [&](int zc) {
            const rsrc_t rl = rs_at(zc - R - 1);
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) Quad<TIn>::load(rl, q1off(k), ps[k]);
        };
        auto do_p12 = [&](int par) {
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) {
                double in4[4], hs[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    zv[k][e] = zv[k][e] + (double)pa[k][e];
                    zv[k][e] = zv[k][e] - (double)ps[k][e];
                    in4[e] = zv[k][e];
                }
                quad_xsums<R>(in4, hs, [](double v, bool lower) {
                    return lower ? dpp_from_lower(v) : dpp_from_upper(v);
                });
                int off, row, qi;
                bool ok;
                p12_geo(k, off, row, qi, ok);
                if (ok) {
                    Hx(par, 0)[row * C::PQ + qi] = make_double2(hs[0], hs[1]);
                    Hx(par, 1)[row * C::PQ + qi] = make_double2(hs[2], hs[3]);
                }
            }
        };
        // prologue: P12(zc_begin) -> Hx[zc_begin & 1]; prefetch step zc_begin
        load_pa(zc_begin);
        load_ps(zc_begin);
        do_p12(zc_begin & 1);
        load_pa(zc_begin + 1);
        load_v5(zc_begin - 1 - R);
        lds_barrier();
        march([&](int i) { load_ps(i + 1); },
              [&](int i, int par) {
                  do_p12(par ^ 1);
                  load_pa(i + 2);
              });
    }
}

// Host: can the v9 kernel take this launch? (radius 1..4, quad-aligned geometry)
template <typename TIn, typename TOut>
inline bool v9_eligible(const GFParams& p, int R) {
    return R >= 1 && R <= 4 && (p.ox0 % 4 == 0) && (p.nx % 4 == 0) && (p.onx % 4 == 0) &&
           (p.in_sy % 4 == 0) && (p.in_sz % 4 == 0) && (p.out_sy % 4 == 0) &&
           (p.out_sz % 4 == 0) && ((uintptr_t)p.in % (4 * sizeof(TIn)) == 0) &&
           ((uintptr_t)p.out % (4 * sizeof(TOut)) == 0);
}

template <int R, typename TIn, typename TOut>
inline hipError_t launch_v9(const GFParams& p0, hipStream_t stream) {
    using C = V9Config<R>;
    GFParams p = p0;
    {
        volatile float one = 1.0f;  // IEEE division on the host: RN(1/W^3)
        p.rcp_w3 = one / (float)C::W3;
    }
    p.tiles_x = (p.onx + C::TX - 1) / C::TX;
    p.tiles_y = (p.ony + C::TY - 1) / C::TY;
    p.nseg = (p.onz + p.zseg - 1) / p.zseg;
    auto kern = gf3d_v9_kernel<R, TIn, TOut>;
    static bool attr_set = false;  // per instantiation
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)C::LDS_BYTES);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const long long nwg = (long long)p.tiles_x * p.tiles_y * p.nseg;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), (size_t)C::LDS_BYTES, stream, p);
    return hipGetLastError();
}

// Fused launch for radius R. gf3d_fused_kernel is the default: on MI355X (2048^3 f32, r=4) it
// runs in 36.4 ms against 51.5 ms for this kernel (tools/timev9, round 1), which is correct
// (max rel. difference 3.3e-7 to the default kernel, tests/test_fused_v9_gpu.py) but loses the
// latency hiding of the two-barrier march: only 1-2 waves per SIMD run the long P3 phase while
// the P12 waves wait at the barrier. ZT_FUSED_V9=1 in the environment selects it where it
// applies (radius 1..4, quad-aligned geometry) for A/B runs.
// zt_set_fused_variant(1) does the same from the C ABI.
inline bool v9_enabled() {
    static const bool env_on = [] {
        const char* e = getenv("ZT_FUSED_V9");
        return e && e[0] == '1';
    }();
    return env_on || fused_variant().load(std::memory_order_relaxed) == 1;
}

template <int R, int TY, int NT, typename TIn, typename TOut>
inline hipError_t launch_fused_auto_v9(const GFParams& p, hipStream_t stream) {
    if constexpr (R >= 1 && R <= 4) {
        if (v9_enabled() && v9_eligible<TIn, TOut>(p, R))
            return launch_v9<R, TIn, TOut>(p, stream);
    }
    return launch_fused_cfg<R, TY, NT, TIn, TOut>(p, stream);
}

}  // namespace zt
