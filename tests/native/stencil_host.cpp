// stencil_host.cpp -- TEST HARNESS: runs the product's stencil functors
// (ocean_model_arch_amd/csrc/sw_stencils.h, the exact code the HIP kernels execute) on the
// host, over the same launch ranges, with every array access bounds-checked.  Used by
// tests/test_stencils_host.py to catch out-of-bounds accesses and arithmetic/write-set bugs on
// the CPU before a kernel reaches the GPU.  Not part of the product (there is no CPU path).
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define OCN_HD
#define OCN_INLINE inline
#define __forceinline__ inline
#define OCN_ATOMIC_INC(p) (++*(p))
#define OCN_ATOMIC_OR(p, v) (*(p) |= (v))
#define OCN_HOST_BOUNDS_CHECK 1
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

template <bool C> static void run_stage(int stage, const ocn_block *b, const Tab<C> &t, const ocn_sw_params *sw,
                                        double tau, int32_t *nbad, bool full)
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
    case OCN_STAGE_HH_INIT: run(range_bnd(b), make_hh_init(b, t, sw->full_free_surface, full)); break;
    case OCN_STAGE_CHECK_SSH_ERR: run(range_interior(b), make_check_ssh_err(b, t, nbad)); break;
    case 11: run(range_fused_a(b, *sw), make_fused_a(b, t, *sw, tau)); break;
    case 12: run(range_interior(b), make_fused_b(b, t, *sw, tau, full)); break;
    case 13: run(range_ring(b), make_fused_c1(b, t, *sw, nbad)); break;
    default: g_oob = -1;
    }
}

// stage: 0..9 = OCN_STAGE_* (reference stages), 10 = check_ssh_err, 11/12/13 = fused A/B/C1.
// bits/rows: the block's compact tables (hst_prepare) or nullptr for the 2-D real(4) arrays;
// full: HhInit::full.  Returns the number of out-of-bounds accesses detected (0 = clean).
extern "C" long hst_stage(int stage, const ocn_block *b, void *const *ptr, const uint8_t *bits, const float *rows,
                          const ocn_sw_params *sw, double tau, int32_t *nbad, int full)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    if (bits) run_stage(stage, b, Tab<true>{ptr, bits, rows, block_rows(b)}, sw, tau, nbad, full != 0);
    else run_stage(stage, b, Tab<false>{ptr}, sw, tau, nbad, full != 0);
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
