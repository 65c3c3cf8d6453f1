"""Many seeds of tests/test_gpu_pair.py's random entry sequences (a bug hunt, GPU): prints the
failures with their op logs."""
import sys
sys.path.insert(0, ".")
import ocean_model_arch_amd as amd
from tests.test_gpu_multirank import _ranks_sequence
from tests.test_gpu_pair import _random_sequence

amd.lib()
OPS = ["step", "step", "step", "step", "tau", "sync", "read", "ssh", "hr", "kc", "uv", "mu", "rhs", "hqn", "opt",
       "opt", "graph"]
lo, hi = int(sys.argv[1]), int(sys.argv[2])
NOPS = int(sys.argv[4]) if len(sys.argv) > 4 else 20
nfail = 0
LAYOUTS = sys.argv[3].split(",") if len(sys.argv) > 3 and sys.argv[3] != "-" else ["pair", "multi", "x2", "tracer", "tracer_x2"]
if len(sys.argv) > 5 and sys.argv[5] == "ranks":
    LAYOUTS = []
for layout in LAYOUTS:
    for seed in range(lo, hi):
        try:
            _random_sequence(amd, layout, seed, OPS, need_path=False, nops=NOPS)
        except AssertionError as e:
            nfail += 1
            print("FAIL", layout, seed, str(e)[:1500], flush=True)
        except Exception as e:   # an OcnError etc.
            nfail += 1
            print("ERROR", layout, seed, type(e).__name__, str(e)[:800], flush=True)
    print("done", layout, flush=True)
print("failures", nfail)


if len(sys.argv) > 5 and sys.argv[5] == "ranks":
    nf = 0
    for tr in (0, 1, 2):
        for seed in range(lo, hi):
            try:
                _ranks_sequence(amd, seed, NOPS, tracers=tr)
            except AssertionError as e:
                nf += 1
                print("FAIL ranks", tr, seed, str(e)[:1500], flush=True)
            except Exception as e:
                nf += 1
                print("ERROR ranks", tr, seed, type(e).__name__, str(e)[:800], flush=True)
        print("done ranks tracers", tr, flush=True)
    print("ranks failures", nf)
