"""A PSy-style time loop for a rocprofv3 HIP API trace (no host sync inside a step).

    rocprofv3 --hip-trace --output-format csv -d DIR -o psy -- python3 scripts/psy_loop.py [N] [BOX]

Runs N iterations of what a reference-shaped host does each time step (model.f90:146 +
shallow_water.f90's syncs as a caller issues them): ocn_ctx_step(ctx, tau, 1) followed by
ocn_ctx_sync of ssh and of the velocities, on one block of a BOX x BOX box -- after one warm-up call
(the one-time checks and table builds).  The markers printed around the loop bracket the region in
the trace: scripts/psy_trace_summary.py counts the synchronising HIP calls inside it.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    box = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    import ocean_model_arch_amd as amd
    m = amd.OceanModel(amd.box_config(box)).init()
    m.step(2).synchronize()   # warm-up: compact tables, coherence and known-constant checks
    for f in ("ssh", "ubrtr", "vbrtr"):
        m.sync(f)
    m.step(1).synchronize()
    t0 = time.perf_counter()
    print(f"LOOP_BEGIN {time.monotonic_ns()}", flush=True)
    for _ in range(n):
        m.step(1)
        for f in ("ssh", "ubrtr", "vbrtr"):
            m.sync(f)
    print(f"LOOP_END {time.monotonic_ns()}", flush=True)
    m.synchronize()
    dt = time.perf_counter() - t0
    print(f"{n} steps of (ocn_ctx_step(1) + 3 x ocn_ctx_sync): {dt / n * 1e3:.3f} ms/step, "
          f"one-pass {m.onepass_active}, tail pending {m.tail_pending}")
    m.close()


if __name__ == "__main__":
    main()
