"""Replays an op log of tests/test_gpu_pair.py's random sequences (prefix by prefix, each from a
fresh model) and prints the first prefix whose fields differ from the oracle (a bug hunt, GPU)."""
import sys
import numpy as np
sys.path.insert(0, ".")
import ocean_model_arch_amd as amd
from tests.test_gpu_parity import OracleTwin

amd.lib()
LAYOUTS = {"pair": (600, (1, 1)), "multi": (100, (1, 1)), "x2": (120, (3, 2)), "tracer": (100, (1, 1)),
           "tracer_x2": (120, (3, 2))}


def run(layout, ops):
    n, blocks = LAYOUTS[layout]
    tracers = 2 if layout.startswith("tracer") else 0
    sw = amd.SWConfig(use_tracers=1, tracer_num=tracers) if tracers else amd.SWConfig()
    m = amd.OceanModel(amd.box_config(n), sw=sw, par=amd.ParallelConfig(*blocks)).init()
    ref = OracleTwin(n, blocks, tracers)

    def bump(nm, f):
        for bl in m.blocks:
            a = f(m.download(bl.k, nm))
            m.upload(bl.k, nm, a)
            ref.upload(bl, nm, a)

    def smooth(a, amp):
        i, j = np.meshgrid(np.arange(a.shape[0]), np.arange(a.shape[1]), indexing="ij")
        return amp * np.exp(-((i - a.shape[0] / 2) ** 2 + (j - a.shape[1] / 2) ** 2) / (a.size / 40.0))

    try:
        m.step(2, check_every=1).synchronize()
        ref.run(2)
        for op in ops:
            op = op.rstrip("*")
            if op.startswith("step") or op.startswith("tau"):
                k = int(op[4:] if op.startswith("step") else op[3:])
                tau = 0.5 if op.startswith("tau") else 1.0
                m.step(k, tau=tau, check_every=1)
                ref.run(k, tau)
            elif op == "sync":
                m.synchronize()
            elif op == "read":
                m.download(0, "ssh")
            elif op == "ssh":
                def f(a):
                    a[a.shape[0] // 2, a.shape[1] // 3] += 1.0e-3
                    return a
                bump("ssh", f)
            elif op == "hr":
                bump("hhq_rest", lambda a: a + smooth(a, 2.0))
            elif op == "uv":
                bump("ubrtr", lambda a: a + smooth(a, 1.0e-4))
            elif op == "mu":
                bump("mu", lambda a: a + smooth(a, 50.0))
            elif op == "rhs":
                bump("RHSx", lambda a: a + smooth(a, 1.0e-7))
            elif op == "hqn":
                bump("hhq_n", lambda a: a + 1.0)
            elif op.startswith("opt-"):
                w, v = op[4:-1], int(op[-1])
                if w == "pair":
                    m.set_pair(v)
                else:
                    {"onepass": m.set_onepass, "multi": m.set_multi, "tracer_step": m.set_tracer_step,
                     "lazy_tail": m.set_lazy_tail, "flip": m.set_flip}[w](bool(v))
            elif op.startswith("graph"):
                m.set_graph(op == "graph1")
            elif op.startswith("kc"):
                m.set_known_constants(op == "kc1")
        return ref.mismatches(m)
    finally:
        m.close()


layout, seq = sys.argv[1], sys.argv[2].split(",")
if len(sys.argv) > 3:   # just this sequence
    print(seq, run(layout, seq)[:6], flush=True)
else:
    for L in range(1, len(seq) + 1):
        bad = run(layout, seq[:L])
        print(L, seq[:L][-3:], bad[:4], flush=True)
        if bad:
            break
