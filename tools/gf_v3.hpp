// gf_v3.hpp — the fused 2.5-D guided-filter kernel, third design (radii 2 and 4).
//
// Same arithmetic as gf3d_fused_kernel (gf_fused.hpp; the reference: guided_filter.rs:117-164):
//   stage 1  U = box_r(v) in f64 (exact), u = RN(RN(U) / count) (Markstein, correctly rounded),
//            s = (v - u)^2, a = s / (s + eps), b = (1 - a) u            (f32, a and b within
//            1 ulp: a = s * rcp(s + eps), b = fma(-a, u, u))
//   stage 2  out = v * mean_r(a) + mean_r(b)                              (f32 window sums)
// but organised around the costs measured on gfx950 (tools/ubench.hip, profiles/r03_ubench.txt):
// a DPP move costs two f32 adds, an f64 add or conversion 1.7, and every LDS write 2.5x a read.
//
// One 512-thread workgroup (8 waves, 2 per SIMD) owns a 64 x 32 output tile and marches along z.
// Three phases per z-step, every wave doing its share of each, one LDS barrier per step with
// double-buffered hand-offs (step i runs A(i+1), B(i), CD(i-1)):
//   A  (lane = 8 consecutive x of one row of the (64+4r) x (32+4r) apron)  running z-window of v
//      in f64, x-window sums from the lane's 8 values and r neighbours on each side (f64 DPP
//      shifts) -> Hx[(32+4r) x (64+2r)] (LDS, f64).
//   B  (lane = 8 rows x 1 column of the (64+2r) x (32+2r) apron)  y-window sums of Hx in f64
//      (8 + 2r rows read per lane: LDS reads are cheaper than f64 DPP shifts), u / a / b, then the
//      y-window sums of (a, b) (own rows + the next lane's prefix sums, DPP folded into the f32
//      adds) -> Yab[32 x (64+2r)] (LDS, float2). Stage 2 runs y before x so one transpose serves
//      both stages (the earlier kernel went rows -> columns -> rows -> columns).
//   CD (lane = 4 consecutive x of one output row)  x-window sums of Yab (three quads read), the
//      z-window over a register ring of the last 2r+1 slice sums (van Herk prefix / suffix
//      blocks), out = v * mean(a) + mean(b), one 16-byte store.
// Per voxel this is ~0.7 of the earlier kernel's VALU cycles and ~0.5 of its LDS cycles.
#pragma once

#include "../zarrs_tools_amd/csrc/gf_fused.hpp"

namespace zt {

template <int R>
struct V3Config {
    static_assert(R == 2 || R == 4, "gf_v3: radii 2 and 4");
    static constexpr int TX = 64, TY = 32, NT = 512, NWAVE = NT / 64;
    static constexpr int W = 2 * R + 1;
    static constexpr int E2X = TX + 4 * R, E2Y = TY + 4 * R;  // v / Zv apron
    static constexpr int E1X = TX + 2 * R, E1Y = TY + 2 * R;  // u / a / b apron
    // A: octets of E2 rows
    static constexpr int NOA = E2X / 8;           // octets per row (10 / 9)
    static constexpr int RPWA = 64 / NOA;         // rows per wave (6 / 7)
    // B: columns x segments of 8 E1 rows
    static constexpr int NSB = (E1Y + 7) / 8;     // segments per column (5 / 5)
    static constexpr int CPWB = 64 / NSB;         // columns per wave (12)
    static constexpr int KB = 8 + 2 * R;          // Hx rows read per B lane
    // CD: 16 quads per output row, 4 rows per wave
    static constexpr int QPR = TX / 4;
    static constexpr int W3 = W * W * W;
    // LDS: f64 pitch = 2 mod 4 (16-byte aligned rows, b64 column reads spread over banks);
    // float2 pitch likewise
    static constexpr int p2m4(int x) { return x + ((2 - x % 4) + 4) % 4; }
    static constexpr int PH = p2m4(E1X);
    static constexpr int PY = p2m4(E1X);
    static constexpr int al(int b) { return (b + 255) / 256 * 256; }
    static constexpr int SZ_HX = al(E2Y * PH * 8);
    static constexpr int SZ_YAB = al(TY * PY * 8);
    static constexpr int SZ_RCP = al((W3 + 1) * 4);
    static constexpr int OFF_HX = 0, OFF_YAB = OFF_HX + 2 * SZ_HX;
    static constexpr int OFF_RCP = OFF_YAB + 2 * SZ_YAB;
    static constexpr int OFF_SINK = OFF_RCP + SZ_RCP;  // writes of inactive lanes
    static constexpr int LDS_BYTES = OFF_SINK + 64 * 16;  // one 16-byte slot per lane
    static_assert(E2X % 8 == 0 && NOA * RPWA <= 64, "A: whole octets per row");
    static_assert((E2Y + RPWA - 1) / RPWA <= NWAVE, "A: rows fit the waves");
    static_assert((E1X + CPWB - 1) / CPWB <= NWAVE, "B: columns fit the waves");
    static_assert(TY / 4 <= NWAVE, "CD: rows fit the waves");
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
};

// own + neighbour(lane + 1), the DPP shift folded into the f32 add (v_add_f32_dpp wave_shl:1);
// lane 63 reads 0 (bound_ctrl).
__device__ __forceinline__ float add_upper(float own, float nb) {
    return own + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, nb),
                                                                    0x130, 0xF, 0xF, true));
}

// MODE 0: interior tiles (the whole apron inside the domain, the tile inside the output box): no
//         masks, window counts depend on z only (wave-uniform, per step);
// MODE 1: other tiles of a quad-aligned geometry (every 4-element quad wholly inside or outside):
//         unmasked quads, per-lane counts and out-of-domain zeroing;
// MODE 2: the remaining tiles: element-wise masked accesses.
template <int R, typename TIn, typename TOut, int MODE>
__global__ __launch_bounds__(512) void gf3d_v3_kernel(GFParams p) {
    using C = V3Config<R>;
    constexpr bool EDGE = MODE == 2;
    constexpr int TX = C::TX, TY = C::TY, W = C::W;
    constexpr int ESZ = (int)sizeof(TIn), OSZ = (int)sizeof(TOut);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* rcp_tab = reinterpret_cast<float*>(smem + C::OFF_RCP);
    char* const sink = smem + C::OFF_SINK;
    auto hx_buf = [&](int i) { return reinterpret_cast<double*>(smem + C::OFF_HX + (i & 1) * C::SZ_HX); };
    auto yab_buf = [&](int i) { return reinterpret_cast<float2*>(smem + C::OFF_YAB + (i & 1) * C::SZ_YAB); };
    const int tid = threadIdx.x;
    for (int c = tid; c <= C::W3; c += C::NT) rcp_tab[c] = c > 0 ? 1.0f / (float)c : 0.0f;
    // zero both hand-off buffers: the pipeline's first steps read buffers no phase has written
    // (their results fall in no emitted window), and zeros keep them finite
    for (int o = tid * 16; o < C::OFF_RCP; o += C::NT * 16)
        *reinterpret_cast<float4*>(smem + o) = make_float4(0.f, 0.f, 0.f, 0.f);

    // ---- XCD-aware block -> (tile, z segment), as gf3d_fused_kernel ---------------------------
    const int nwg = gridDim.x, b = blockIdx.x;
    const int lid = (nwg % 8 == 0) ? (b % 8) * (nwg / 8) + b / 8 : b;
    const int gtx = MODE ? p.tiles_x : p.itx1 - p.itx0;
    const int gty = MODE ? p.tiles_y : p.ity1 - p.ity0;
    const int ntiles = gtx * gty;
    const int seg = lid / ntiles;
    int t = lid % ntiles, tile_x, tile_y;
    {
        const int stx = GF_STX, sty = GF_STY;
        const int full_y = gty / sty * sty, per_srow = gtx * sty;
        if (t < full_y * gtx) {
            const int sr = t / per_srow, r = t % per_srow, full_x = gtx / stx * stx;
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
    if constexpr (MODE) {
        if (tile_x >= p.itx0 && tile_x < p.itx1 && tile_y >= p.ity0 && tile_y < p.ity1) return;
    } else {
        tile_x += p.itx0;
        tile_y += p.ity0;
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
    auto rs_at = [&](int z) -> rsrc_t {  // descriptor of input plane z (0 records outside)
        const bool ok = (unsigned)(z - zlo) < (unsigned)zspan;
        return make_rsrc(in_base + (ok ? (int64_t)(z - p.in_z0) * sstride : 0), ok ? slice_bytes : 0u);
    };
    const bool xy_interior = x0 - 2 * R >= 0 && x0 + TX + 2 * R <= nx && y0 - 2 * R >= 0 &&
                             y0 + TY + 2 * R <= ny;
    constexpr float kW3 = (float)C::W3;
    const float rcp_w3 = p.rcp_w3;

    const int wave = tid >> 6, lane = tid & 63;
    // ---- A lane: E2 row ra, octet oa ---------------------------------------------------------
    const int ra = wave * C::RPWA + lane / C::NOA, oa = lane % C::NOA;
    const bool a_act = lane < C::RPWA * C::NOA && ra < C::E2Y;
    const int a_gx = x0 - 2 * R + 8 * oa, a_gy = y0 - 2 * R + ra;
    int a_off[2], a_mask[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        int m = 0;
        if (a_act && a_gy >= 0 && a_gy < ny) {
#pragma unroll
            for (int e = 0; e < 4; ++e) m |= ((unsigned)(a_gx + 4 * h + e) < (unsigned)nx) ? (1 << e) : 0;
        }
        a_mask[h] = m;
        a_off[h] = (EDGE ? a_act : m == 0xF) ? (a_gy * sy + a_gx + 4 * h) * ESZ : kBadOff;
    }
    auto load_oct = [&](rsrc_t r, float (&v)[8]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float q[4];
            if constexpr (EDGE) load_quad_masked<TIn>(r, a_off[h], a_mask[h], q);
            else Quad<TIn>::load(r, a_off[h], q);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[4 * h + e] = q[e];
        }
    };
    // ---- B lane: column cb, segment sb --------------------------------------------------------
    const int cb = wave * C::CPWB + lane / C::NSB, sb = lane % C::NSB;
    const bool b_act = lane < C::CPWB * C::NSB && cb < C::E1X;
    const int b_gx = x0 - R + cb, b_gy0 = y0 - R + 8 * sb;
    // ---- CD lane: output row tc, quad qc ------------------------------------------------------
    const int tc = wave * 4 + lane / C::QPR, qc = lane % C::QPR;
    const int d_ox = x0 + 4 * qc, d_oy = y0 + tc;
    int d_mask = 0;
    if (d_oy < oy_end) {
#pragma unroll
        for (int e = 0; e < 4; ++e) d_mask |= (d_ox + e < ox_end) ? (1 << e) : 0;
    }
    const int d_in_off = (EDGE ? (d_oy < ny && d_ox < nx) : d_mask == 0xF) ? (d_oy * sy + d_ox) * ESZ : kBadOff;
    const int d_out_off =
        (EDGE ? d_mask != 0 : d_mask == 0xF) ? ((d_oy - p.oy0) * osy + (d_ox - p.ox0)) * OSZ : kBadOff;

    // ---- march bounds -------------------------------------------------------------------------
    const int zc_begin = zo_begin - R;  // first stage-1 slice any output of the segment needs
    // step i runs A(i+1), B(i), CD(i-1) and stores output slice i-1-R
    const int i_begin = zc_begin - 1;
    const int n_steps = ((zo_end + R) - i_begin + 1 + W - 1) / W * W;

    // Zv(zc_begin - 1): the z-window of v seeded over [zc_begin-1-R, zc_begin-1+R] clamped
    double zv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) zv[e] = 0.0;
    {
        const int za = max(zc_begin - 1 - R, 0), zb_ = min(zc_begin - 1 + R, nz - 1);
        for (int z = za; z <= zb_; ++z) {
            float v[8];
            load_oct(rs_at(z), v);
#pragma unroll
            for (int e = 0; e < 8; ++e) zv[e] += (double)v[e];
        }
    }
    // prefetched inputs of the next step
    float pa[8], pl[8];  // A: entering / leaving octets
    float vb[8];         // B: v at the lane's 8 E1 points of its next slice
    float vd[4];         // CD: v at the lane's output quad of its next output slice
    auto load_b = [&](rsrc_t r) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int gy = b_gy0 + k;
            bool ok = b_act;
            if constexpr (EDGE) ok = ok && (unsigned)b_gx < (unsigned)nx && (unsigned)gy < (unsigned)ny;
            else ok = ok && 8 * sb + k < C::E1Y;
            vb[k] = Buf<TIn>::load(r, opaque(ok ? (gy * sy + b_gx) * ESZ : kBadOff));
        }
    };
    auto load_d = [&](rsrc_t r) {
        if constexpr (EDGE) {
            int m = 0;
            if (d_oy < ny) {
#pragma unroll
                for (int e = 0; e < 4; ++e) m |= (d_ox + e < nx) ? (1 << e) : 0;
            }
            load_quad_masked<TIn>(r, d_in_off, m, vd);
        } else {
            Quad<TIn>::load(r, d_in_off, vd);
        }
    };

    // stage-2 z ring (van Herk / Gil-Werman blocks, slot = compile-time position in the block)
    f2 ring[W][4], pre[4];
#pragma unroll
    for (int s = 0; s < W; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) ring[s][j] = (f2){0.0f, 0.0f};
#pragma unroll
    for (int j = 0; j < 4; ++j) pre[j] = (f2){0.0f, 0.0f};

    // ---- phase A: z-window update + x-window sums -> Hx -------------------------------------
    auto phase_a = [&](double* hx) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            zv[e] = zv[e] + (double)pa[e];
            zv[e] = zv[e] - (double)pl[e];
        }
        double in[8 + 2 * R], hs[8];
#pragma unroll
        for (int e = 0; e < R; ++e) in[e] = dpp_from_lower(zv[8 - R + e]);
#pragma unroll
        for (int e = 0; e < 8; ++e) in[R + e] = zv[e];
#pragma unroll
        for (int e = 0; e < R; ++e) in[R + 8 + e] = dpp_from_upper(zv[e]);
        slide_sums_f64<R, 8>(in, hs);
        // center column c = 8 oa + k -> Hx column c - R (pairs: R even, 16-byte aligned)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int col = 8 * oa + 2 * h - R;
            const bool ok = a_act && col >= 0 && col + 1 < C::E1X;
            double* dst = ok ? hx + ra * C::PH + col : reinterpret_cast<double*>(sink + 16 * lane);
            *reinterpret_cast<double2*>(dst) = make_double2(hs[2 * h], hs[2 * h + 1]);
        }
    };

    // ---- phase B: y-window of Hx, u / a / b, y-window of (a, b) -> Yab ------------------------
    auto phase_b = [&](const double* hx, float2* yab, int zc) {
        // (all lanes run the arithmetic; inactive ones read row 0 and write to the sink)
        double h[C::KB], U[8];
        const int colr = b_act ? cb : 0;
#pragma unroll
        for (int i = 0; i < C::KB; ++i) {
            const int row = min(8 * sb + i, C::E2Y - 1);
            h[i] = hx[row * C::PH + colr];
        }
        slide_sums_f64<R, 8>(h, U);
        f2 ab[8];
        const bool interior = xy_interior && zc - R >= 0 && zc + R < nz;  // wave-uniform
        if (interior) {
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                const f2 Uf = {(float)U[k], (float)U[k + 1]};
                const f2 cnt = {kW3, kW3}, rc = {rcp_w3, rcp_w3};
                const f2 q = Uf * rc;
                const f2 r = pk_fma(-q, cnt, Uf);
                const f2 u = pk_fma(r, rc, q);
                const f2 vv = {vb[k], vb[k + 1]};
                f2 s = vv - u;
                s = s * s;
                const f2 den = s + (f2){eps, eps};
                const f2 y = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
                const f2 a = s * y;
                const f2 bb = pk_fma(-a, u, u);
                ab[k] = (f2){a.x, bb.x};
                ab[k + 1] = (f2){a.y, bb.y};
            }
        } else {
            const bool zin = zc >= 0 && zc < nz;
            const int cz = clamped_count(min(max(zc, 0), nz - 1), nz, R);
            const bool xin = (unsigned)b_gx < (unsigned)nx;
            const int cx = clamped_count(b_gx, nx, R);
#pragma unroll
            for (int k = 0; k < 8; k += 2) {
                int c0 = max(clamped_count(b_gy0 + k, ny, R) * cx * cz, 1);
                int c1 = max(clamped_count(b_gy0 + k + 1, ny, R) * cx * cz, 1);
                c0 = min(c0, C::W3);
                c1 = min(c1, C::W3);
                const f2 Uf = {(float)U[k], (float)U[k + 1]};
                const f2 cnt = {(float)c0, (float)c1}, rc = {rcp_tab[c0], rcp_tab[c1]};
                const f2 q = Uf * rc;
                const f2 r = pk_fma(-q, cnt, Uf);
                const f2 u = pk_fma(r, rc, q);
                const f2 vv = {vb[k], vb[k + 1]};
                f2 s = vv - u;
                s = s * s;
                const f2 den = s + (f2){eps, eps};
                const f2 y = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
                const f2 a = s * y;
                const f2 bb = pk_fma(-a, u, u);
                // zero outside the domain: the clamped window sums of stage 2
                const bool ok0 = zin && xin && (unsigned)(b_gy0 + k) < (unsigned)ny;
                const bool ok1 = zin && xin && (unsigned)(b_gy0 + k + 1) < (unsigned)ny;
                ab[k] = ok0 ? (f2){a.x, bb.x} : (f2){0.f, 0.f};
                ab[k + 1] = ok1 ? (f2){a.y, bb.y} : (f2){0.f, 0.f};
            }
        }
        // rows past the E1 apron (last segment) hold no (a, b)
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (8 * (C::NSB - 1) + k >= C::E1Y && sb == C::NSB - 1) ab[k] = (f2){0.f, 0.f};
        // y-window sums of (a, b): row t = 8 sb + k needs E1 rows t .. t + 2R, i.e. own rows
        // k .. 7 and the next segment's first k + 2R - 7 rows (its prefix sums, by DPP)
        f2 prefix[8], suffix[8];  // prefix[m] = ab[0..m], suffix[m] = ab[m..7]
        prefix[0] = ab[0];
#pragma unroll
        for (int m = 1; m < 8; ++m) prefix[m] = prefix[m - 1] + ab[m];
        suffix[7] = ab[7];
#pragma unroll
        for (int m = 6; m >= 0; --m) suffix[m] = ab[m] + suffix[m + 1];
        static_for<0, 8>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            f2 own;
            if constexpr (k + 2 * R >= 7) {
                own = suffix[k];
            } else {
                own = ab[k];
#pragma unroll
                for (int j = 1; j <= 2 * R; ++j) own = own + ab[k + j];
            }
            float ya = own.x, yb = own.y;
            if constexpr (k + 2 * R >= 8) {
                const f2 nb = prefix[k + 2 * R - 8];
                ya = add_upper(ya, nb.x);
                yb = add_upper(yb, nb.y);
            }
            const int trow = 8 * sb + k;
            const bool ok = b_act && trow < TY;
            float2* dst = ok ? yab + trow * C::PY + cb : reinterpret_cast<float2*>(sink + 16 * lane);
            *dst = make_float2(ya, yb);
        });
    };

    // ---- phase CD: x-window of Yab, z ring, output --------------------------------------------
    auto phase_cd = [&](const float2* yab, int zo, rsrc_t ro, auto slot_c) {
        constexpr int P = decltype(slot_c)::value;
        constexpr int NIN = 4 + 2 * R;
        f2 in[NIN], q5[4];
        const float2* src = yab + tc * C::PY + 4 * qc;
#pragma unroll
        for (int j = 0; j < NIN; j += 2) {
            const float4 f = *reinterpret_cast<const float4*>(src + j);
            in[j] = (f2){f.x, f.y};
            in[j + 1] = (f2){f.z, f.w};
        }
        core_window_sums<R, 4>(in, q5);
        f2 AB[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            pre[j] = (P == 0) ? q5[j] : pre[j] + q5[j];
            if constexpr (P == W - 1) AB[j] = pre[j];
            else AB[j] = ring[(P + 1) % W][j] + pre[j];
            ring[P][j] = q5[j];
        }
        if constexpr (P == W - 1) {
#pragma unroll
            for (int s = W - 2; s >= 0; --s)
#pragma unroll
                for (int j = 0; j < 4; ++j) ring[s][j] = ring[s][j] + ring[s + 1][j];
        }
        const bool interior = xy_interior && zo - R >= 0 && zo + R < nz;  // wave-uniform
        float o[4];
        if (interior) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f2 m = AB[j] * (f2){rcp_w3, rcp_w3};
                o[j] = __fadd_rn(__fmul_rn(vd[j], m.x), m.y);
            }
        } else {
            const int zq = min(max(zo, 0), nz - 1);
            const int cyz = clamped_count(min(d_oy, ny - 1), ny, R) * clamped_count(zq, nz, R);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int cnt = min(max(clamped_count(min(d_ox + j, nx - 1), nx, R) * cyz, 1), C::W3);
                const float rr = rcp_tab[cnt];
                const f2 m = AB[j] * (f2){rr, rr};
                o[j] = __fadd_rn(__fmul_rn(vd[j], m.x), m.y);
            }
        }
        if constexpr (EDGE) {
            store_quad_masked<TOut>(o, ro, d_out_off, d_mask);
        } else {
            float oo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) oo[j] = from_f32<TOut>(o[j]);
            Quad<TOut>::store(oo, ro, opaque(d_out_off));
        }
    };

    // ---- prologue -----------------------------------------------------------------------------
    // step i = i_begin: A(i+1 = zc_begin) needs entering zc_begin+R, leaving zc_begin-1-R
    load_oct(rs_at(zc_begin + R), pa);
    load_oct(rs_at(zc_begin - 1 - R), pl);
    load_b(rs_at(i_begin));
    load_d(rs_at(i_begin - 1 - R));
    lds_barrier();  // rcp table and zeroed buffers

    // ---- the march, unrolled by W so the ring slot of CD is a compile-time constant ----------
    for (int i0 = i_begin; i0 < i_begin + n_steps; i0 += W) {
        static_for<0, W>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int i = i0 + k;
            // CD(i-1): ring slot of slice i-1 relative to i_begin - 1
            const int zs = i - 1 - R;  // output slice stored this step
            const rsrc_t ro = make_rsrc(out_base + (int64_t)(zs - p.oz0) * osstride,
                                        (unsigned)(zs - zo_begin) < (unsigned)(zo_end - zo_begin)
                                            ? oslice_bytes : 0u);
            phase_cd(yab_buf(i - 1), zs, ro, std::integral_constant<int, (k + W - 1) % W>{});
            phase_a(hx_buf(i + 1));
            phase_b(hx_buf(i), yab_buf(i), i);
            // next step's inputs: A(i+2): entering i+2+R, leaving i+1-R; B(i+1); CD(i): v(i-R)
            load_oct(rs_at(i + 2 + R), pa);
            load_oct(rs_at(i + 1 - R), pl);
            load_b(rs_at(i + 1));
            load_d(rs_at(i - R));
            lds_barrier();
        });
    }
}

template <int R, typename TIn, typename TOut, bool EDGE>
inline hipError_t launch_v3_variant(const GFParams& p, long long nwg, hipStream_t stream) {
    using C = V3Config<R>;
    auto kern = gf3d_v3_kernel<R, TIn, TOut, EDGE>;
    if (hipError_t e = allow_dynamic_lds((const void*)kern, C::LDS_BYTES, attr_devices<decltype(kern)>()))
        return e;
    if (nwg <= 0) return hipSuccess;
    if (nwg > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(C::NT), (size_t)C::LDS_BYTES, stream, p);
    return hipGetLastError();
}

template <int R, typename TIn, typename TOut>
inline hipError_t launch_v3_cfg(const GFParams& p0, hipStream_t stream) {
    using C = V3Config<R>;
    GFParams p = p0;
    {
        volatile float one = 1.0f;
        p.rcp_w3 = one / (float)C::W3;
    }
    p.tiles_x = (p.onx + C::TX - 1) / C::TX;
    p.tiles_y = (p.ony + C::TY - 1) / C::TY;
    p.nseg = (p.onz + p.zseg - 1) / p.zseg;
    const bool quad_ok = (p.ox0 % 4 == 0) && (p.nx % 4 == 0) && (p.onx % 4 == 0) &&
                         (p.in_sy % 4 == 0) && (p.in_sz % 4 == 0) && (p.out_sy % 4 == 0) &&
                         (p.out_sz % 4 == 0) && ((uintptr_t)p.in % (4 * sizeof(TIn)) == 0) &&
                         ((uintptr_t)p.out % (4 * sizeof(TOut)) == 0);
    if (quad_ok) {
        p.itx0 = 0; p.itx1 = p.tiles_x;
        p.ity0 = 0; p.ity1 = p.tiles_y;
    } else {
        interior_tiles(p.ox0, p.ox0 + p.onx, p.nx, C::TX, R, 4, p.tiles_x, p.itx0, p.itx1);
        interior_tiles(p.oy0, p.oy0 + p.ony, p.ny, C::TY, R, 0, p.tiles_y, p.ity0, p.ity1);
    }
    const long long n_int = (long long)(p.itx1 - p.itx0) * (p.ity1 - p.ity0);
    const long long n_all = (long long)p.tiles_x * p.tiles_y;
    hipError_t e = hipSuccess;
    if (n_int > 0) e = launch_v3_variant<R, TIn, TOut, false>(p, n_int * p.nseg, stream);
    if (e == hipSuccess && n_all > n_int)
        e = launch_v3_variant<R, TIn, TOut, true>(p, n_all * p.nseg, stream);
    return e;
}

}  // namespace zt
