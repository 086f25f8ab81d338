"""`python tests/bench_fake_ranks.py --gpus N ...` behaves as `python bench.py
--gpus N ...` started without a launcher: bench.main() spawns the N rank
processes itself (bench.launch_ranks re-runs this same script).  In every rank
(RANK set) the device entry points are first swapped for the CPU-oracle
stand-ins of test_dist_gloo.py, so the whole N-rank orchestration runs on CPU.
Used by test_dist_gloo.py::test_bench_self_launch_world2; not a test module."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "0g-ec-gpu_amd")]

if __name__ == "__main__":
    if "RANK" in os.environ:
        from test_dist_gloo import _install_device_fakes

        _install_device_fakes(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]),
                              fail_rank=int(os.environ["FAKE_FAIL_RANK"]) if "FAKE_FAIL_RANK" in os.environ else None)
    import bench

    bench.main()
