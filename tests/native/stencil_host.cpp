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

// stage: 0..9 = OCN_STAGE_* (reference stages), 10 = check_ssh_err, 11/12/13 = fused A/B/C1.
// Returns the number of out-of-bounds accesses detected (0 = clean).
extern "C" long hst_stage(int stage, const ocn_block *b, void *const *ptr, const ocn_sw_params *sw, double tau,
                          int32_t *nbad)
{
    g_oob = 0;
    ocn_host_limit = (unsigned)(b->pitch * (int64_t)(b->bnd_y2 - b->bnd_y1 + 1));
    switch (stage) {
    case OCN_STAGE_SW_UPDATE_SSH: run(range_interior(b), make_sw_update_ssh(b, ptr, tau)); break;
    case OCN_STAGE_HH_UPDATE: run(range_bnd(b), make_hh_update(b, ptr)); break;
    case OCN_STAGE_UV_TRANS_VORT: run(range_interior(b), make_uv_trans_vort(b, ptr)); break;
    case OCN_STAGE_UV_TRANS: run(range_interior(b), make_uv_trans(b, ptr)); break;
    case OCN_STAGE_STRESS_COMPONENTS: run(range_interior(b), make_stress_components(b, ptr)); break;
    case OCN_STAGE_UV_DIFF2: run(range_interior(b), make_uv_diff2(b, ptr)); break;
    case OCN_STAGE_SW_UPDATE_UV: run(range_interior(b), make_sw_update_uv(b, ptr, tau)); break;
    case OCN_STAGE_SW_NEXT_STEP: run(range_ring(b), make_sw_next_step(b, ptr, sw->time_smooth)); break;
    case OCN_STAGE_HH_SHIFT: run(range_ring(b), make_hh_shift(b, ptr, sw->time_smooth)); break;
    case OCN_STAGE_HH_INIT: run(range_bnd(b), make_hh_init(b, ptr, sw->full_free_surface)); break;
    case OCN_STAGE_CHECK_SSH_ERR: {
        CheckSshErr k{geo(b), (const float *)ptr[ocn_field_slot(OCN_LU)], (const double *)ptr[ocn_field_slot(OCN_SSH)],
                      (int *)nbad};
        run(range_interior(b), k);
        break;
    }
    case 11: run(range_fused_a(b, *sw), make_fused_a(b, ptr, *sw, tau)); break;
    case 12: run(range_interior(b), make_fused_b(b, ptr, *sw, tau)); break;
    case 13: run(range_ring(b), make_fused_c1(b, ptr, *sw, nbad)); break;
    default: return -1;
    }
    return g_oob;
}
