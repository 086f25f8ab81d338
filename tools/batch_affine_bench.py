"""Runs tools/batch_affine_bench (build it first: see the .hip header) on
4096 BLS12-381 G1 bases from the CPU oracle (dev tool).
Usage: python tools/batch_affine_bench.py [out.log]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import coracle as co  # noqa: E402

B = co.gen_bases(0, 0x5151, 0x2323, 4096)
assert B.shape == (4096, 12)
with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
    B.tofile(f)
    path = f.name
out = subprocess.run([os.path.join(ROOT, "tools", "batch_affine_bench"), path], capture_output=True, text=True,
                     timeout=600)
os.unlink(path)
sys.stdout.write(out.stdout)
sys.stderr.write(out.stderr)
sys.exit(out.returncode)
