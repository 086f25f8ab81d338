"""A plain-C program compiles against include/ecgpu.h and links
libecgpu.so (gcc, no Python in the call path): the FFI shape a Rust / Go / C
prover binds.  CPU: build + the no-device path.  GPU: an FFT
and an MSM through the C program, checked against the CPU oracle."""
import os
import subprocess

import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po
from conftest import ROOT


def build_demo(tmp_path):
    exe = str(tmp_path / "abi_demo")
    libdir = os.path.dirname(ecgpu.LIB_PATH)
    subprocess.check_call(["gcc", "-O2", "-Wall", "-Werror", "-std=c11", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "abi_demo.c"), "-o", exe, "-L", libdir, "-lecgpu",
                           f"-Wl,-rpath,{libdir}"])
    return exe


def test_c_program_builds_and_runs(tmp_path):
    exe = build_demo(tmp_path)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "gfx950" in out.stdout and "/opt/rocm" in out.stdout
    if ecgpu.lib().ecg_device_count() == 0:
        assert "no-device path ok" in out.stdout


@pytest.mark.gpu
def test_c_program_fft_and_msm(tmp_path):
    exe = build_demo(tmp_path)
    f = po.BLS12_381_FR
    rng = po.Xoshiro256ss(0xC0DE)
    log_n, m = 12, 3000
    data = co.u64arr([f.to_mont(rng.field_element(f)) for _ in range(1 << log_n)], 4)
    om = co.u64arr([f.to_mont(f.omega(1 << log_n))], 4)[0]
    bases = co.gen_bases(0, 91, 92, m, 8)
    sc = co.u64arr([rng.field_element(f) for _ in range(m)], 4)
    inp = tmp_path / "in.bin"
    outp = tmp_path / "out.bin"
    np.concatenate([np.array([log_n, m], dtype=np.uint64), om, data.ravel(), bases.ravel(), sc.ravel()]).tofile(inp)
    r = subprocess.run([exe, str(inp), str(outp)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(outp, dtype=np.uint64)
    fft_out = got[:4 << log_n].reshape(-1, 4)
    msm_out = got[4 << log_n:]
    assert (fft_out == co.serial_fft(0, data, om, log_n)).all()
    want = co.multiexp_cpu(0, bases, sc, nthreads=8)
    assert (co.jac_to_affine(0, msm_out) == co.jac_to_affine(0, want)).all()
