// gf_role.hpp — the fused 2.5-D guided filter with the work split into two wave roles (round 6).
//
// Same arithmetic as gf3d_fused_kernel (gf_fused.hpp; guided_filter.rs:117-164): stage 1 (the
// exact window sums of v -> u, a, b) and stage 2 (the box means of a and b -> out) over a 64 x 32
// output tile that marches along z. What changes is who does what:
//
//   stage-1 waves (8 of 16): P12 (running z-window of v, x-window by DPP -> Hx) and P3 (y-window
//     of Hx -> U -> u, a, b -> Lab). VALU-heavy (f64 / int32 sums, DPP, the pointwise chain).
//   stage-2 waves (the other 8): P4 (x-window of Lab -> Hab) and P5 (y-window of Hab, z-window
//     from a register ring, out = v * mean(a) + mean(b)). LDS-heavy.
//
// In gf3d_fused_kernel every wave runs every phase, so all 16 waves are in the same phase between
// two barriers and its LDS-heavy heads and VALU-heavy bodies do not overlap: a z-step costs about
// the sum of the VALU (~1700 SIMD-cycles) and LDS (~1900) time. Here each SIMD
// holds two waves of each role, so an LDS-heavy stage-2 wave issues beside a VALU-heavy stage-1
// wave. Each wave also carries only its own role's persistent state (stage 1: the f64 z-window and
// the prefetched quads; stage 2: the (a, b) z-ring), so the registers freed pay for more outputs
// per stage-2 thread (4, against 2): P5 reads Hab 3x instead of 5x per output.
//
// The hand-offs are double-buffered in LDS (Hx, Lab, Hab: 149 KB at r = 4), so one barrier per
// step suffices: step i runs P3(i) + P12(i + 1) on the stage-1 waves and P4(i - 1) + P5(i - 2) on
// the stage-2 waves, every phase reading the buffer written in the previous step.
//
// Scope: quad-aligned geometry (the mode-1 grid of gf3d_fused_kernel: every tile with unmasked
// 16-byte accesses, out-of-domain quads through kBadOff, per-lane clamped counts), even r <= 4,
// f32 / u16 / u8 inputs. Other cases keep gf3d_fused_kernel.
#pragma once

#include "gf_fused.hpp"

#ifndef GF_ROLE_S1_LOW
#define GF_ROLE_S1_LOW 1  // stage-1 role on waves 0-7 (1) or on waves 8-15 (0)
#endif
#ifndef GF_ROLE_PRIO
#define GF_ROLE_PRIO 0  // 1: the stage-1 waves run at s_setprio 1 (static, set once)
#endif
#ifndef GF_ROLE_K3
#define GF_ROLE_K3 6  // P3 outputs per stage-1 thread (a column segment of the y-window)
#endif
#ifndef GF_ROLE_K4
#define GF_ROLE_K4 8  // P4 outputs per item (a row segment of the (a, b) x-window)
#endif
#ifndef GF_ROLE_P4FIRST
#define GF_ROLE_P4FIRST 1  // stage-2 waves: P4 before P5 within a step
#endif
#ifndef GF_ROLE_SKIP
#define GF_ROLE_SKIP 0  // timing only (wrong output): 1 = stage-2 waves skip their phases, 2 = stage-1
#endif
#ifndef GF_ROLE_ORDER
#define GF_ROLE_ORDER 0  // stage-1 step order: 0 P12 pass 0 / P3 / other passes; 1 P12 joint, P3; 2 P3, P12 joint
#endif
#ifndef GF_ROLE_PF
#define GF_ROLE_PF 2  // stage-1 slices prefetched this many steps ahead (1 or 2)
#endif

namespace zt {

template <int R, int HXB>
struct RoleConfig {
    static constexpr int TX = 64, TY = 32, NT = 1024;
    static constexpr int NW = 8;  // waves per role
    static constexpr int W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    using G = GFConfig<R, TY, NT, HXB>;
    // P12: one lane per quad of an E2 row, whole rows per wave (x neighbours by DPP)
    static constexpr int NQ1X = E2X / 4;
    static constexpr int RPW = 64 / NQ1X;
    static constexpr int NQP1 = (E2Y + RPW * NW - 1) / (RPW * NW);
    static constexpr int NB = (R + 3) / 4;
    // P3: column segments of K3 rows
    static constexpr int K3 = GF_ROLE_K3;
    static constexpr int S3 = (E1Y + K3 - 1) / K3;
    static constexpr int N3 = E1X * S3;
    // P4: row segments of K4 outputs
    static constexpr int K4 = GF_ROLE_K4;
    static constexpr int S4 = TX / K4;
    static constexpr int N4 = E1Y * S4;
    // P5: K5 consecutive rows of one column per stage-2 thread
    static constexpr int K5 = TX * TY / (64 * NW);
    static constexpr int W3 = W * W * W;
    // Hx rows hold E1 columns -4 .. E1X+3 at offset HXS = 4: the P12 lanes of a row's first and
    // last quad write their out-of-apron columns into that margin instead of branching around
    // the store; the 64 - RPW * NQ1X lanes past a wave's rows write a dummy row.
    static constexpr int HXS = 4;
    static constexpr int PH = HXB == 8 ? G::p2m4(E1X + 2 * HXS) : G::ph4(E1X + 2 * HXS);
    static constexpr int PA = G::PA, PB = G::PB;
    static constexpr int HX_ROWS = S3 * K3 + 2 * R;  // rows P3 reads (past E2Y: never stored)
    static constexpr int P12_ROWS = NQP1 * NW * RPW;  // rows the P12 lanes address
    static constexpr int HX_DUMMY = HX_ROWS > P12_ROWS ? HX_ROWS : P12_ROWS;
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_HX = al((HX_DUMMY + 1) * PH * HXB);
    static constexpr int SZ_LAB = al(S3 * K3 * PA * 8);  // P3's last segment may pass E1Y
    static constexpr int SZ_HAB = al(E1Y * PB * 8);
    static constexpr int SZ_RCP = al((W3 + 1) * 4);
    static constexpr int OFF_HX = 0;                       // two buffers each
    static constexpr int OFF_LAB = OFF_HX + 2 * SZ_HX;
    static constexpr int OFF_HAB = OFF_LAB + 2 * SZ_LAB;
    static constexpr int OFF_RCP = OFF_HAB + 2 * SZ_HAB;
    static constexpr int LDS_BYTES = OFF_RCP + SZ_RCP;
    static_assert(R % 2 == 0 && R <= 4, "even radii up to 4 (quad-aligned aprons)");
    static_assert(RPW >= 1 && E2X % 4 == 0, "an E2 row is whole quads within one wave");
    static_assert(N3 <= 64 * NW && N4 <= 64 * NW, "one item per thread per phase");
    static_assert(K3 % 2 == 0 && TY % K5 == 0 && TX % K4 == 0, "work splits");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

template <int R, typename TIn>
inline constexpr bool role_supported() {
    return (R == 2 || R == 4) &&
           (std::is_same<TIn, float>::value || std::is_same<TIn, uint16_t>::value ||
            std::is_same<TIn, uint8_t>::value);
}

template <int R, typename TIn, typename TOut>
__global__ __launch_bounds__(1024) void gf3d_role_kernel(GFParams p) {
    using SA = typename S1<TIn>::acc;  // stage-1 window sums (exact)
    using SI = typename S1<TIn>::in;   // loaded stage-1 values
    using C = RoleConfig<R, S1<TIn>::HXB>;
    constexpr int TX = C::TX, TY = C::TY, W = C::W;
    constexpr int K3 = C::K3, K4 = C::K4, K5 = C::K5;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* const rcp_tab = reinterpret_cast<float*>(smem + C::OFF_RCP);
    for (int c = threadIdx.x; c <= C::W3; c += C::NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;

    // XCD-aware block -> tile, as gf3d_fused_kernel (mode 1: the whole tile grid)
    const int nwg = gridDim.x;
    const int bidx = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (bidx % 8) * (nwg / 8) + bidx / 8 : bidx;
    const int gtx = p.tiles_x, gty = p.tiles_y;
    const int ntiles = gtx * gty;
    const int seg = lid / ntiles;
    int tile_x, tile_y;
    {
        int t = lid % ntiles;
        const int stx = GF_STX, sty = GF_STY;
        const int full_y = gty / sty * sty;
        const int per_srow = gtx * sty;
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
    const int x0 = p.ox0 + tile_x * TX;
    const int y0 = p.oy0 + tile_y * TY;
    const int zo_begin = p.oz0 + seg * p.zseg;
    const int zo_end = min(zo_begin + p.zseg, p.oz0 + p.onz);
    const int nz = p.nz, ny = p.ny, nx = p.nx;
    const int sy = (int)p.in_sy;  // 32-bit: slices < 2 GiB (host check)
    const uint32_t slice_bytes = (uint32_t)((int64_t)(p.ny - 1) * p.in_sy + p.nx) * ESZ;
    const char* in_base = static_cast<const char*>(p.in);
    const int zlo = p.zlo, zspan = p.zhi - p.zlo;
    const int64_t sstride = p.in_sz * ESZ;
    auto rs_in = [&](int64_t off, int z) {  // slice z at byte offset off; 0-record outside [zlo, zhi)
        return make_rsrc(in_base + off, (unsigned)(z - zlo) < (unsigned)zspan ? slice_bytes : 0u);
    };
    auto slice_off = [&](int z) { return (int64_t)(z - p.in_z0) * sstride; };

    const int zc_begin = zo_begin - R, zc_end = zo_end + R;  // stage-1 slices of this march
    // Step i runs P3(i) + P12(i+1) (stage 1) and P4(i-1) + P5(i-2) (stage 2); P5(c) emits
    // out(c - R), so the last output slice zo_end - 1 is emitted at step zc_end + 1. The step count
    // is padded to a multiple of the unroll (every ring slot and buffer index a constant).
    constexpr int PF = GF_ROLE_PF;
    constexpr int UN = 2 * W * (PF == 2 ? 1 : 1);  // even (double buffers) and a multiple of W
    const int n_steps = (zc_end + 2 - zc_begin + UN - 1) / UN * UN;

    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bool stage1 = GF_ROLE_S1_LOW ? wave < C::NW : wave >= C::NW;
    const int rt = (int)threadIdx.x - (stage1 == (bool)GF_ROLE_S1_LOW ? 0 : 64 * C::NW);  // 0..511

    if (stage1) {
        // =============================== stage 1: P12 + P3 ===================================
        if constexpr (GF_ROLE_PRIO) __builtin_amdgcn_s_setprio(1);
        const int w1 = rt >> 6, l1 = rt & 63;
        int q1off[C::NQP1], hxa[C::NQP1];  // quad offsets; Hx element index of the lane's writes
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k) {
            const int row = (k * C::NW + w1) * C::RPW + l1 / C::NQ1X, cq = l1 % C::NQ1X;
            const bool lane = l1 < C::RPW * C::NQ1X;
            const bool valid = lane && row < C::E2Y;
            const int gx = x0 - 2 * R + 4 * cq, gy = y0 - 2 * R + row;
            // quad-aligned geometry: a quad lies wholly inside or outside the domain
            const bool in = valid && gy >= 0 && gy < ny && gx >= 0 && gx < nx;
            q1off[k] = in ? (gy * sy + gx) * ESZ : kBadOff;
            // Hx column of the quad's first x-window output: 4 cq - R (+ HXS); rows past E2Y
            // are never read as stage-1 rows
            hxa[k] = lane ? row * C::PH + 4 * cq - R + C::HXS : C::HX_DUMMY * C::PH + 4 * (l1 & 15);
        }
        SA zv[C::NQP1][4];
#pragma unroll
        for (int k = 0; k < C::NQP1; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) zv[k][e] = (SA)0;
        {  // seed: Zv(zc_begin - 1) = sum over [zc_begin-1-R, zc_begin-1+R] clamped to [0, nz)
            const int za = max(zc_begin - 1 - R, 0), zb_ = min(zc_begin - 1 + R, nz - 1);
            for (int z = za; z <= zb_; ++z) {
                const rsrc_t rs = rs_in(slice_off(z), z);
#pragma unroll
                for (int k = 0; k < C::NQP1; ++k) {
                    SI v[4];
                    Quad<TIn>::load(rs, q1off[k], v);
#pragma unroll
                    for (int e = 0; e < 4; ++e) zv[k][e] += (SA)v[e];
                }
            }
        }
        SI pa[PF][C::NQP1][4], ps[PF][C::NQP1][4];
        auto load_p1 = [&](auto bc, rsrc_t ra, rsrc_t rs) {  // entering, leaving
            constexpr int b = decltype(bc)::value;
#pragma unroll
            for (int k = 0; k < C::NQP1; ++k) {
                Quad<TIn>::load(ra, q1off[k], pa[b][k]);
                Quad<TIn>::load(rs, q1off[k], ps[b][k]);
            }
        };
        // P12(c), pass k: the z-window of v (exact, running) and its x-window sums on the E2
        // apron -> Hx; every lane stores (margin columns and the dummy row absorb the rest)
        auto do_p12 = [&](auto kc, auto bc, auto hbc) {
            constexpr int k = decltype(kc)::value;
            constexpr int b = decltype(bc)::value;
            SA* const Hx = reinterpret_cast<SA*>(smem + C::OFF_HX + decltype(hbc)::value * C::SZ_HX);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                zv[k][e] = zv[k][e] + (SA)pa[b][k][e];
                zv[k][e] = zv[k][e] - (SA)ps[b][k][e];
            }
            constexpr int NB = C::NB;
            SA win[4 * (2 * NB + 1)];
#pragma unroll
            for (int e = 0; e < 4; ++e) win[4 * NB + e] = zv[k][e];
#pragma unroll
            for (int n = 1; n <= NB; ++n)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    win[4 * (NB - n) + e] = dpp_from_lower(win[4 * (NB - n + 1) + e]);
                    win[4 * (NB + n) + e] = dpp_from_upper(win[4 * (NB + n - 1) + e]);
                }
            SA vin[4 + 2 * R], hs[4];
#pragma unroll
            for (int j = 0; j < 4 + 2 * R; ++j) vin[j] = win[4 * NB - R + j];
            slide_sums_exact<R, 4>(vin, hs);
            if constexpr (C::G::HXB_ == 4 && R % 4 == 0) {
                *reinterpret_cast<int4*>(Hx + hxa[k]) = make_int4(hs[0], hs[1], hs[2], hs[3]);
            } else if constexpr (C::G::HXB_ == 4) {
                *reinterpret_cast<int2*>(Hx + hxa[k]) = make_int2(hs[0], hs[1]);
                *reinterpret_cast<int2*>(Hx + hxa[k] + 2) = make_int2(hs[2], hs[3]);
            } else {
                *reinterpret_cast<double2*>(Hx + hxa[k]) = make_double2(hs[0], hs[1]);
                *reinterpret_cast<double2*>(Hx + hxa[k] + 2) = make_double2(hs[2], hs[3]);
            }
        };
        // All P12 passes stage by stage (z-update, DPP, window sums, stores of every pass in
        // turn): independent chains side by side for the two stage-1 waves of a SIMD to issue.
        auto do_p12_joint = [&](auto bc, auto hbc) {
            constexpr int b = decltype(bc)::value;
            SA* const Hx = reinterpret_cast<SA*>(smem + C::OFF_HX + decltype(hbc)::value * C::SZ_HX);
            constexpr int NB = C::NB, NQ = C::NQP1;
#pragma unroll
            for (int k = 0; k < NQ; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    zv[k][e] = zv[k][e] + (SA)pa[b][k][e];
                    zv[k][e] = zv[k][e] - (SA)ps[b][k][e];
                }
            SA win[NQ][4 * (2 * NB + 1)];
#pragma unroll
            for (int k = 0; k < NQ; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) win[k][4 * NB + e] = zv[k][e];
#pragma unroll
            for (int n = 1; n <= NB; ++n)
#pragma unroll
                for (int k = 0; k < NQ; ++k)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        win[k][4 * (NB - n) + e] = dpp_from_lower(win[k][4 * (NB - n + 1) + e]);
                        win[k][4 * (NB + n) + e] = dpp_from_upper(win[k][4 * (NB + n - 1) + e]);
                    }
            SA hs[NQ][4];
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                SA vin[4 + 2 * R];
#pragma unroll
                for (int j = 0; j < 4 + 2 * R; ++j) vin[j] = win[k][4 * NB - R + j];
                slide_sums_exact<R, 4>(vin, hs[k]);
            }
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                if constexpr (C::G::HXB_ == 4 && R % 4 == 0) {
                    *reinterpret_cast<int4*>(Hx + hxa[k]) =
                        make_int4(hs[k][0], hs[k][1], hs[k][2], hs[k][3]);
                } else if constexpr (C::G::HXB_ == 4) {
                    *reinterpret_cast<int2*>(Hx + hxa[k]) = make_int2(hs[k][0], hs[k][1]);
                    *reinterpret_cast<int2*>(Hx + hxa[k] + 2) = make_int2(hs[k][2], hs[k][3]);
                } else {
                    *reinterpret_cast<double2*>(Hx + hxa[k]) = make_double2(hs[k][0], hs[k][1]);
                    *reinterpret_cast<double2*>(Hx + hxa[k] + 2) = make_double2(hs[k][2], hs[k][3]);
                }
            }
        };
        // P3(c): y-window (exact) of Hx -> U; u = RN(U)/count, s = (v-u)^2, a, b -> Lab.
        // Positions outside the domain get count 0: rcp_tab[0] = 0 and the Markstein division
        // then gives u = 0, and their v reads 0 (kBadOff, or a zero-record slice), so s = 0 and
        // a = 0 / eps = 0, b = 0: the zero padding that makes stage 2's window sums the clamped
        // sums, with no per-lane select (eps > 0: host check). Counts of the K3 rows are packed
        // 8 bits each (cx * cy <= (2R+1)^2). Threads past the N3 items repeat the last segment's
        // item of their column (same values, same Lab cells): no branch.
        constexpr int NP3 = K3 / 2;
        const int col3 = rt % C::E1X, sg3 = min(rt / C::E1X, C::S3 - 1);
        const int gx3 = x0 - R + col3, gy30 = y0 - R + sg3 * K3;
        const bool xin3 = gx3 >= 0 && gx3 < nx;
        const int cx3 = xin3 ? clamped_count(gx3, nx, R) : 0;
        unsigned cxy3[(K3 + 3) / 4];
        int voff3[K3];
#pragma unroll
        for (int q = 0; q < (K3 + 3) / 4; ++q) cxy3[q] = 0u;
#pragma unroll
        for (int k = 0; k < K3; ++k) {
            const int gy = gy30 + k;
            const bool in = xin3 && gy >= 0 && gy < ny;
            cxy3[k / 4] |= (unsigned)(in ? cx3 * clamped_count(gy, ny, R) : 0) << (8 * (k % 4));
            voff3[k] = in ? (gy * sy + gx3) * ESZ : kBadOff;
        }
        float vc[K3];
        auto load_p3v = [&](rsrc_t r) {
#pragma unroll
            for (int k = 0; k < K3; ++k) vc[k] = Buf<TIn>::load(r, opaque(voff3[k]));
        };
        const int hx3 = (sg3 * K3) * C::PH + col3 + C::HXS;  // P3's first Hx element
        auto p3_load = [&](auto hbc, SA (&vin)[K3 + 2 * R]) {
            const SA* src = reinterpret_cast<const SA*>(smem + C::OFF_HX + decltype(hbc)::value * C::SZ_HX) + hx3;
#pragma unroll
            for (int j = 0; j < K3 + 2 * R; ++j) vin[j] = src[j * C::PH];
        };
        float2* const lab3 = reinterpret_cast<float2*>(smem + C::OFF_LAB) + (sg3 * K3) * C::PA + col3;
        auto do_p3 = [&](int zc, auto hbc, const SA (&vin)[K3 + 2 * R]) {
            constexpr int hb = decltype(hbc)::value;
            SA U[K3];
            slide_sums_exact<R, K3>(vin, U);
            f2 Uf[NP3], vv[NP3], fc[NP3], rc[NP3], a[NP3], bb[NP3];
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                Uf[k] = (f2){(float)U[2 * k], (float)U[2 * k + 1]};
                vv[k] = (f2){vc[2 * k], vc[2 * k + 1]};
            }
            const int cz = (unsigned)zc < (unsigned)nz ? clamped_count(zc, nz, R) : 0;  // uniform
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                const int c0 = cmul(__builtin_amdgcn_ubfe(cxy3[(2 * k) / 4], 8 * ((2 * k) % 4), 8), cz);
                const int c1 =
                    cmul(__builtin_amdgcn_ubfe(cxy3[(2 * k + 1) / 4], 8 * ((2 * k + 1) % 4), 8), cz);
                fc[k] = (f2){(float)c0, (float)c1};
                rc[k] = (f2){rcp_tab[c0], rcp_tab[c1]};
            }
            // the pointwise chain of gf3d_fused_kernel (guided_filter.rs:126-137)
            f2 q[NP3], rr[NP3], u[NP3], sq[NP3], den[NP3], y[NP3];
#pragma unroll
            for (int k = 0; k < NP3; ++k) q[k] = Uf[k] * rc[k];
#pragma unroll
            for (int k = 0; k < NP3; ++k) rr[k] = pk_fma(-q[k], fc[k], Uf[k]);
#pragma unroll
            for (int k = 0; k < NP3; ++k) u[k] = pk_fma(rr[k], rc[k], q[k]);
#pragma unroll
            for (int k = 0; k < NP3; ++k) sq[k] = vv[k] - u[k];
#pragma unroll
            for (int k = 0; k < NP3; ++k) sq[k] = sq[k] * sq[k];
#pragma unroll
            for (int k = 0; k < NP3; ++k) den[k] = sq[k] + (f2){p.eps, p.eps};
#pragma unroll
            for (int k = 0; k < NP3; ++k)
                y[k] = (f2){__builtin_amdgcn_rcpf(den[k].x), __builtin_amdgcn_rcpf(den[k].y)};
#pragma unroll
            for (int k = 0; k < NP3; ++k) q[k] = sq[k] * y[k];
#pragma unroll
            for (int k = 0; k < NP3; ++k) rr[k] = pk_fma(-den[k], q[k], sq[k]);
#pragma unroll
            for (int k = 0; k < NP3; ++k) a[k] = pk_fma(rr[k], y[k], q[k]);
#pragma unroll
            for (int k = 0; k < NP3; ++k) bb[k] = ((f2){1.0f, 1.0f} - a[k]) * u[k];
            // (rows past E1Y land in the buffer's spare rows and are never read)
            float2* const lab = lab3 + hb * (C::SZ_LAB / 8);
#pragma unroll
            for (int k = 0; k < NP3; ++k) {
                lab[(2 * k) * C::PA] = make_float2(a[k].x, bb[k].x);
                lab[(2 * k + 1) * C::PA] = make_float2(a[k].y, bb[k].y);
            }
        };
        static_assert(C::SZ_LAB % 8 == 0, "Lab buffer stride in float2");

        // ---- prologue: P12(zc_begin) -> Hx[0]; prefetches ------------------------------------
        using B0 = std::integral_constant<int, 0>;
        using BL = std::integral_constant<int, PF - 1>;
        load_p1(BL{}, rs_in(slice_off(zc_begin + R), zc_begin + R),
                rs_in(slice_off(zc_begin - R - 1), zc_begin - R - 1));
        load_p3v(rs_in(slice_off(zc_begin), zc_begin));
        static_for<0, C::NQP1>([&](auto kc) { do_p12(kc, BL{}, B0{}); });
        load_p1(B0{}, rs_in(slice_off(zc_begin + 1 + R), zc_begin + 1 + R),
                rs_in(slice_off(zc_begin - R), zc_begin - R));
        if constexpr (PF == 2)
            load_p1(BL{}, rs_in(slice_off(zc_begin + 2 + R), zc_begin + 2 + R),
                    rs_in(slice_off(zc_begin + 1 - R), zc_begin + 1 - R));
        lds_barrier();

        // step i: v of slice i+1 (P3's next), entering slice i+1+PF+R, leaving i+PF-R. The two
        // phases are independent within a step: P3's LDS reads are issued first, P12's first
        // pass runs while they land, then P3's arithmetic, then the other passes.
        int zv3 = zc_begin + 1;
        int64_t ov3 = slice_off(zv3);
        const int64_t off_e = (int64_t)(PF + R) * sstride, off_l = (int64_t)(PF - R - 1) * sstride;
        for (int i0 = zc_begin; i0 < zc_begin + n_steps; i0 += UN) {
            static_for<0, UN>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const int i = i0 + k;
                using BK = std::integral_constant<int, k % PF>;
                using HR = std::integral_constant<int, k & 1>;        // Hx / Lab of slice i
                using HW = std::integral_constant<int, (k + 1) & 1>;  // Hx of slice i + 1
                if constexpr (GF_ROLE_SKIP != 2) {
                    SA vin3[K3 + 2 * R];
                    p3_load(HR{}, vin3);
                    if constexpr (GF_ROLE_ORDER == 1) {  // P12 passes jointly, then P3
                        do_p12_joint(BK{}, HW{});
                        do_p3(i, HR{}, vin3);
                    } else if constexpr (GF_ROLE_ORDER == 2) {  // P3, then P12 jointly
                        do_p3(i, HR{}, vin3);
                        do_p12_joint(BK{}, HW{});
                    } else {  // P12 pass 0, P3, the other passes
                        do_p12(std::integral_constant<int, 0>{}, BK{}, HW{});
                        do_p3(i, HR{}, vin3);
                        static_for<1, C::NQP1>([&](auto pc) { do_p12(pc, BK{}, HW{}); });
                    }
                }
                load_p3v(rs_in(ov3, zv3));
                load_p1(BK{}, rs_in(ov3 + off_e, zv3 + PF + R), rs_in(ov3 + off_l, zv3 + PF - R - 1));
                lds_barrier();
                ++zv3;
                ov3 += sstride;
            });
        }
    } else {
        // =============================== stage 2: P4 + P5 =====================================
        const int col5 = rt % TX, seg5 = rt / TX;
        const int ox = x0 + col5, oyb = y0 + seg5 * K5;
        const int ox_end = p.ox0 + p.onx, oy_end = p.oy0 + p.ony;
        const int osy = (int)p.out_sy;
        const uint32_t oslice_bytes = (uint32_t)((int64_t)(p.ony - 1) * p.out_sy + p.onx) * OSZ;
        const char* out_base = static_cast<const char*>(p.out);
        const int64_t osstride = p.out_sz * OSZ;
        const unsigned nzo = (unsigned)(zo_end - zo_begin);
        int voff[K5], ooff[K5];
        f2 ring[W][K5], pre[K5];
        float v5[K5];
#pragma unroll
        for (int j = 0; j < K5; ++j) {
            const int oy = oyb + j;
            const bool ok = ox < ox_end && oy < oy_end;
            voff[j] = ok ? (oy * sy + ox) * ESZ : kBadOff;
            ooff[j] = ok ? ((oy - p.oy0) * osy + (ox - p.ox0)) * OSZ : kBadOff;
            pre[j] = (f2){0.0f, 0.0f};
            v5[j] = 0.0f;
        }
#pragma unroll
        for (int s = 0; s < W; ++s)
#pragma unroll
            for (int j = 0; j < K5; ++j) ring[s][j] = (f2){0.0f, 0.0f};
        // the x * y window counts of the K5 outputs, 8 bits each (<= (2R+1)^2; clamped
        // coordinates keep the table index valid where the store drops)
        unsigned cxy5 = 0u;
        {
            const int cx = clamped_count(min(ox, nx - 1), nx, R);
#pragma unroll
            for (int j = 0; j < K5; ++j)
                cxy5 |= (unsigned)(cx * clamped_count(min(oyb + j, ny - 1), ny, R)) << (8 * j);
        }
        static_assert(K5 <= 4, "packed counts");

        auto load_p5v = [&](rsrc_t r) {
#pragma unroll
            for (int j = 0; j < K5; ++j) v5[j] = Buf<TIn>::load(r, opaque(voff[j]));
        };
        // P4(c): x-window sums of the (a, b) rows of Lab -> Hab
        const int item4 = rt;
        auto do_p4 = [&](auto hbc) {
            constexpr int hb = decltype(hbc)::value;
            // whole waves past the items branch around the phase (scalar test)
            if (__builtin_amdgcn_readfirstlane(item4 >> 6) * 64 >= C::N4) return;
            // lanes past the items repeat the last one (same values, same cells): no branch
            const int it = min(item4, C::N4 - 1);
            const int row = it % C::E1Y, sg = it / C::E1Y;
            const float2* lab = reinterpret_cast<const float2*>(smem + C::OFF_LAB + hb * C::SZ_LAB);
            const float4* src = reinterpret_cast<const float4*>(lab + row * C::PA + sg * K4);
            f2 vin[K4 + 2 * R], vout[K4];
#pragma unroll
            for (int j = 0; j < (K4 + 2 * R) / 2; ++j) {
                const float4 f = src[j];
                vin[2 * j] = (f2){f.x, f.y};
                vin[2 * j + 1] = (f2){f.z, f.w};
            }
            core_window_sums<R, K4>(vin, vout);
            float2* hab = reinterpret_cast<float2*>(smem + C::OFF_HAB + hb * C::SZ_HAB);
            float4* dst = reinterpret_cast<float4*>(hab + row * C::PB + sg * K4);
#pragma unroll
            for (int j = 0; j < K4 / 2; ++j)
                dst[j] = make_float4(vout[2 * j].x, vout[2 * j].y, vout[2 * j + 1].x, vout[2 * j + 1].y);
        };
        // P5(c): y-window of Hab -> slice sums; z-window (van Herk blocks of W in the ring);
        // out(c - R) = v * mean(a) + mean(b) with two roundings (guided_filter.rs:144-162)
        auto do_p5 = [&](int c, auto slot_c, auto hbc, rsrc_t ro) {
            constexpr int P = decltype(slot_c)::value;
            constexpr int hb = decltype(hbc)::value;
            const f2* src = reinterpret_cast<const f2*>(smem + C::OFF_HAB + hb * C::SZ_HAB) +
                            (seg5 * K5) * C::PB + col5;
            f2 vin[K5 + 2 * R];
#pragma unroll
            for (int j = 0; j < K5 + 2 * R; ++j) vin[j] = src[j * C::PB];
            f2 s2[K5];
            core_window_sums<R, K5>(vin, s2);
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
            const int cz = clamped_count(min(max(c - R, 0), nz - 1), nz, R);  // uniform
#pragma unroll
            for (int j = 0; j < K5; ++j) {
                const float r = rcp_tab[cmul(__builtin_amdgcn_ubfe(cxy5, 8 * j, 8), cz)];
                const f2 q = AB[j] * (f2){r, r};
                const float o = __fadd_rn(__fmul_rn(v5[j], q.x), q.y);  // v*=ma; v+=mb
                Buf<TOut>::store(from_f32<TOut>(o), ro, opaque(ooff[j]));
            }
        };

        // prologue: v for P5(zc_begin - 2) (its output slice lies before the segment: dropped)
        int zs = zc_begin - 2 - R;  // output slice of this step's P5
        int64_t vsoff = slice_off(zs);
        int64_t os = (int64_t)(zs - p.oz0) * osstride;
        load_p5v(rs_in(vsoff, zs));
        lds_barrier();
        for (int i0 = zc_begin; i0 < zc_begin + n_steps; i0 += UN) {
            static_for<0, UN>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                const int i = i0 + k;
                const rsrc_t ro = make_rsrc(out_base + os, (unsigned)(zs - zo_begin) < nzo ? oslice_bytes : 0u);
                if constexpr (GF_ROLE_SKIP != 1) {
                    if constexpr (GF_ROLE_P4FIRST) do_p4(std::integral_constant<int, (k + 1) & 1>{});
                    do_p5(i - 2, std::integral_constant<int, (k + 2 * W - 2) % W>{},
                          std::integral_constant<int, k & 1>{}, ro);
                    if constexpr (!GF_ROLE_P4FIRST) do_p4(std::integral_constant<int, (k + 1) & 1>{});
                }
                ++zs;
                vsoff += sstride;
                os += osstride;
                load_p5v(rs_in(vsoff, zs));
                lds_barrier();
            });
        }
    }
}

// Quad-aligned geometry (launch_fused_cfg's mode-1 condition): every 4-element quad of a global
// access lies wholly inside or outside the domain and the output box.
template <int R, typename TIn, typename TOut>
inline bool fused_quad_ok(const GFParams& p) {
    return (p.ox0 % 4 == 0) && (R % 2 == 0) && (p.nx % 4 == 0) && (p.onx % 4 == 0) &&
           (p.in_sy % 4 == 0) && (p.in_sz % 4 == 0) && (p.out_sy % 4 == 0) &&
           (p.out_sz % 4 == 0) && ((uintptr_t)p.in % (4 * sizeof(TIn)) == 0) &&
           ((uintptr_t)p.out % (4 * sizeof(TOut)) == 0);
}

template <int R, typename TIn, typename TOut>
inline hipError_t launch_role(const GFParams& p0, hipStream_t stream) {
    using C = RoleConfig<R, S1<TIn>::HXB>;
    GFParams p = p0;
    p.tiles_x = (p.onx + C::TX - 1) / C::TX;
    p.tiles_y = (p.ony + C::TY - 1) / C::TY;
    p.nseg = (p.onz + p.zseg - 1) / p.zseg;
    p.itx0 = p.itx1 = p.ity0 = p.ity1 = 0;
    auto kern = gf3d_role_kernel<R, TIn, TOut>;
    if (hipError_t e = allow_dynamic_lds((const void*)kern, C::LDS_BYTES, attr_devices<decltype(kern)>()))
        return e;
    const long long nwg = (long long)p.tiles_x * p.tiles_y * p.nseg;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), (size_t)C::LDS_BYTES, stream, p);
    return hipGetLastError();
}

#ifndef GF_ROLE
#define GF_ROLE 0  // the role-split kernel for the cases it covers (0: gf3d_fused_kernel always)
#endif

// The fused launch of gf_fused_r<R>.hip: the role-split kernel where it applies.
template <int R, int TY, int NT, typename TIn, typename TOut>
inline hipError_t launch_fused_pick(const GFParams& p, hipStream_t s) {
    if constexpr (GF_ROLE && TY == 32 && NT == 1024 && role_supported<R, TIn>()) {
        // eps > 0: its zero padding relies on a = 0 / eps = 0 outside the domain
        if (fused_quad_ok<R, TIn, TOut>(p) && p.eps > 0.0f) return launch_role<R, TIn, TOut>(p, s);
    }
    return launch_fused_cfg<R, TY, NT, TIn, TOut>(p, s);
}

}  // namespace zt
