// stencil_host.cpp -- TEST HARNESS: runs the product's stencil functors
// (ocean_model_arch_amd/csrc/sw_stencils.h, the exact code the HIP kernels execute) on the
// host, over the same launch ranges, with every array access bounds-checked.  Used by
// tests/test_stencils_host.py to catch out-of-bounds accesses and arithmetic/write-set bugs on
// the CPU before a kernel reaches the GPU.  Not part of the product (there is no CPU path).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define OCN_HD
#define OCN_INLINE inline
#define __forceinline__ inline
#define OCN_ATOMIC_INC(p) (++*(p))
#define OCN_ATOMIC_OR(p, v) (*(p) |= (v))
#define OCN_HOST_BOUNDS_CHECK 1
#define OCN_WAVE_ALL(p) (p)
#include "../../ocean_model_arch_amd/csrc/sw_stencils.h"

static long g_oob = 0;
namespace ocn {
unsigned ocn_host_limit = 0;
void ocn_host_oob(unsigned i)
{
    if (g_oob++ < 5) fprintf(stderr, "stencil_host: out-of-bounds element index %u (limit %u)\n", i, ocn_host_limit);
}
}  // namespace ocn

using namespace ocn;

template <class K> static void run(const Range &r, const K &k)
{
    for (int n = r.n0; n <= r.n1; ++n)
        for (int m = r.m0; m <= r.m1; ++m) k(m, n);
}

// part 0 = whole range, 1 = frame (frame_rects, in the device kernel's point order), 2 = inner
template <class K> static void run_part(const Range &r, const Range &inner, int part, const K &k)
{
    if (part == 2) { run(range_clip(r, inner), k); return; }
    if (part == 1) {
        const Rects q = frame_rects(r, inner);
        for (int t = 0, n = q.total(); t < n; ++t) { int m, nn; frame_point(q, t, m, nn); k(m, nn); }
        return;
    }
    run(r, k);
}

template <bool C> static void run_stage(int stage, const ocn_block *b, const Tab<C> &t, const ocn_sw_params *sw,
                                        double tau, int32_t *nbad, bool full, bool reuse, int part)
{
    switch (stage) {
    case OCN_STAGE_SW_UPDATE_SSH: run(range_interior(b), make_sw_update_ssh(b, t, tau)); break;
    case OCN_STAGE_HH_UPDATE: run(range_bnd(b), make_hh_update(b, t)); break;
    case OCN_STAGE_UV_TRANS_VORT: run(range_interior(b), make_uv_trans_vort(b, t)); break;
    case OCN_STAGE_UV_TRANS: run(range_interior(b), make_uv_trans(b, t)); break;
    case OCN_STAGE_STRESS_COMPONENTS: run(range_interior(b), make_stress_components(b, t)); break;
    case OCN_STAGE_UV_DIFF2: run(range_interior(b), make_uv_diff2(b, t)); break;
    case OCN_STAGE_SW_UPDATE_UV: run(range_interior(b), make_sw_update_uv(b, t, tau)); break;
    case OCN_STAGE_SW_NEXT_STEP: run(range_ring(b), make_sw_next_step(b, t, sw->time_smooth)); break;
    case OCN_STAGE_HH_SHIFT: run(range_ring(b), make_hh_shift(b, t, sw->time_smooth)); break;
    case OCN_STAGE_HH_INIT:   // as the fused C2 launch (KHhInit); full = true is the reference kernel
        run_part(range_bnd(b), inner_interior_shrunk(b), part, KHhInit<C>{*b, t, sw->full_free_surface, full});
        break;
    case OCN_STAGE_CHECK_SSH_ERR: run(range_interior(b), make_check_ssh_err(b, t, nbad)); break;
    // the fused launch functors exactly as sw_kernels.hip passes them (stage functors built inside)
    case 11:
        run_part(range_fused_a(b, *sw, reuse), inner_interior_shrunk(b), part, KFusedA<C>{*b, t, *sw, tau, reuse});
        break;
    case 12:
        run_part(range_interior(b), inner_interior_shrunk(b), part, KFusedB<C>{*b, t, *sw, tau, full, reuse});
        break;
    case 13: run_part(range_ring(b), range_interior(b), part, KFusedC1<C>{*b, t, *sw, nbad}); break;
    default: g_oob = -1;
    }
}

// stage: 0..9 = OCN_STAGE_* (reference stages), 10 = check_ssh_err, 11/12/13 = fused A/B/C1.
// bits/rows: the block's compact tables (hst_prepare) or nullptr for the 2-D real(4) arrays;
// flags: bit 0 = FusedB / HhInit `full`, bit 1 = fused A/B "reuse"; part: the halo-overlap
// split (fused A/B/C1, hh_init).  Returns the number of out-of-bounds accesses (0 = clean).
extern "C" long hst_stage(int stage, const ocn_block *b, void *const *ptr, int nptr, const uint8_t *bits,
                          const float *rows, const ocn_sw_params *sw, double tau, int32_t *nbad, int flags, int part)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    const bool full = flags & 1, reuse = (flags & 2) != 0;
    if (bits)
        run_stage(stage, b, make_tab<true>(ptr, nptr, bits, rows, block_rows(b)), sw, tau, nbad, full, reuse, part);
    else run_stage(stage, b, make_tab<false>(ptr, nptr, nullptr, nullptr, 0), sw, tau, nbad, full, reuse, part);
    return g_oob;
}

// Frame/inner split of a range: 1 if every point of r is in exactly one of the two parts.
extern "C" int hst_split_ok(int m0, int m1, int n0, int n1, int i0, int i1, int j0, int j1)
{
    const Range r{m0, m1, n0, n1}, inner{i0, i1, j0, j1};
    const int w = m1 - m0 + 1, h = n1 - n0 + 1;
    if (w <= 0 || h <= 0) return frame_rects(r, inner).total() == 0;
    std::vector<int> hit((size_t)w * h, 0);
    auto mark = [&](int m, int n) {
        if (m < m0 || m > m1 || n < n0 || n > n1) { hit[0] += 100; return; }
        ++hit[(size_t)(m - m0) + (size_t)(n - n0) * w];
    };
    const Rects q = frame_rects(r, inner);
    for (int t = 0, n = q.total(); t < n; ++t) { int m, nn; frame_point(q, t, m, nn); mark(m, nn); }
    const Range i = range_clip(r, inner);
    for (int n = i.n0; n <= i.n1; ++n)
        for (int m = i.m0; m <= i.m1; ++m) mark(m, n);
    for (int v : hit)
        if (v != 1) return 0;
    return 1;
}

// Tracer stage (OCN_TSTAGE_*) of tracer k: ptr must hold the tracer slots (flux_x, flux_y,
// ff1/ff1p/ff1n per tracer) after the SW ones.
extern "C" long hst_tracer(int stage, const ocn_block *b, void *const *ptr, int nptr, const uint8_t *bits,
                           const float *rows, int k, double tau, double ts, double factor_mu)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    auto go = [&](const auto &t) {
        using T = std::decay_t<decltype(t)>;
        constexpr bool C = std::is_same_v<T, Tab<true>>;
        switch (stage) {   // the launch functors of sw_kernels.hip launch_tracer
        case OCN_TSTAGE_TRAN_DIFF_FLUXES: run(range_interior(b), KTranDiffFluxes<C>{*b, t, factor_mu}); break;
        case OCN_TSTAGE_TRAN_DIFF_TRACER: run(range_interior(b), KTranDiffTracer<C>{*b, t, tau}); break;
        case OCN_TSTAGE_TRACER_NEXT_STEP: run(range_ring(b), KTracerNextStep<C>{*b, t, ts}); break;
        default: g_oob = -1;
        }
    };
    if (bits) go(make_tab<true>(ptr, nptr, bits, rows, block_rows(b), k));
    else go(make_tab<false>(ptr, nptr, nullptr, nullptr, 0, k));
    return g_oob;
}

// The tracer step of tracer k (sw_kernels.hip launch_tracer_step: KTracerStep over the interior),
// its ffn / filtered ffp into ffn_out / ffp_out; own = the halo points neighbour blocks own.
extern "C" long hst_tracer_step(const ocn_block *b, void *const *ptr, int nptr, const uint8_t *bits,
                                const float *rows, int k, double tau, double ts, unsigned own, double *ffn_out,
                                double *ffp_out)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    if (bits) run(range_interior(b), KTracerStep<true>{*b, make_tab<true>(ptr, nptr, bits, rows, block_rows(b), k),
                                                        tau, ts, own, ffn_out, ffp_out});
    else run(range_interior(b), KTracerStep<false>{*b, make_tab<false>(ptr, nptr, nullptr, nullptr, 0, k), tau, ts,
                                                   own, ffn_out, ffp_out});
    return g_oob;
}

// The compact tables of a block (Prepare, thread grid = bnd range); returns the OCN_COMPACT_* flags.
extern "C" int hst_prepare(const ocn_block *b, void *const *ptr, uint8_t *bits, float *rows)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    int flags = 0;
    run(range_bnd(b), make_prepare(b, ptr, bits, rows, &flags));
    return g_oob ? -1 : flags;
}
