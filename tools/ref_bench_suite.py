"""Run bench.reference_bench_suite alone (dev tool): python tools/ref_bench_suite.py CURVE..."""
import os, sys, json, time
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [os.path.join(ROOT, "0g-ec-gpu_amd"), os.path.join(ROOT, "oracle"), ROOT]
import bench, ecgpu, coracle as co
prog = ecgpu.program(ecgpu.Device(0))
for cv in sys.argv[1:]:
    t = time.time()
    r = bench.reference_bench_suite(prog, cv, 0, 16, co)
    print(cv, f"{time.time()-t:.1f} s", json.dumps({k: r[k] for k in ("amt", "amt_window_grid")}), flush=True)
