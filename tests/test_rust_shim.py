"""The Rust shim (integration/rust/) against the C ABI it binds (include/ecgpu.h).

No Rust toolchain exists in the image, so the shim cannot be compiled here;
these checks keep it from drifting from the header: every header function is
declared in ffi.rs with the same arity, the same pointer / scalar kind per
argument and the same return kind, every header constant has the same value,
and every ffi:: call in amd.rs names a declared function with its arity.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ecgpu.h")
FFI = os.path.join(ROOT, "integration", "rust", "ffi.rs")
AMD = os.path.join(ROOT, "integration", "rust", "amd.rs")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", s, flags=re.S)


def _split_args(s):
    s = s.strip()
    if s in ("", "void"):
        return []
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "(<[":
            depth += 1
        elif ch in ")>]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    out.append(cur.strip())
    return out


def _c_kind(decl):
    """'ptr', 'int' (32-bit int / enum-like), 'u32', 'usize', 'void', 'fnptr'."""
    if "ecg_abort_cb" in decl:
        return "fnptr"
    if "*" in decl:
        return "ptr"
    t = decl.split()
    base = " ".join(x for x in t if x not in ("const",))
    if base.startswith("size_t"):
        return "usize"
    if base.startswith("uint32_t"):
        return "u32"
    if base.startswith("int"):
        return "int"
    if base.startswith("void"):
        return "void"
    raise AssertionError(f"unhandled C type in {decl!r}")


def _rs_kind(ty):
    ty = ty.strip()
    if ty == "ecg_abort_cb":
        return "fnptr"
    if ty.startswith("*"):
        return "ptr"
    return {"c_int": "int", "u32": "u32", "usize": "usize", "": "void"}[ty]


def header_functions():
    src = _strip_c_comments(open(HEADER).read())
    funcs = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w\s\*]*?)\b(ecg_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.M | re.S):
        ret, name, args = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        if ret.startswith("typedef"):
            continue
        funcs[name] = (_c_kind(ret + " x"), [_c_kind(a) for a in _split_args(args)])
    return funcs


def ffi_functions():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    funcs = {}
    for m in re.finditer(r"pub fn (ecg_\w+)\s*\((.*?)\)\s*(->\s*([^;]+))?;", block, flags=re.S):
        name, args, ret = m.group(1), " ".join(m.group(2).split()), (m.group(4) or "").strip()
        kinds = [_rs_kind(a.split(":", 1)[1]) for a in _split_args(args)]
        funcs[name] = (_rs_kind(ret), kinds)
    return funcs


def test_header_parses():
    funcs = header_functions()
    assert len(funcs) >= 40 and "ecg_msm" in funcs and "ecg_fft_many" in funcs


def test_every_header_function_declared_with_matching_signature():
    h, r = header_functions(), ffi_functions()
    assert sorted(h) == sorted(r), (set(h) ^ set(r))
    for name, (ret, args) in h.items():
        rret, rargs = r[name]
        # const char * returns are pointers on both sides; int returns are c_int
        assert rret == ret, f"{name}: return {rret} vs header {ret}"
        assert rargs == args, f"{name}: args {rargs} vs header {args}"


def test_constants_match_header():
    src = _strip_c_comments(open(HEADER).read())
    consts = {m.group(1): int(m.group(2)) for m in
              re.finditer(r"#define\s+(ECG_\w+)\s+\(?(-?\d+)\)?", src)}
    rs = {m.group(1): int(m.group(2)) for m in
          re.finditer(r"pub const (ECG_\w+): c_int = (-?\d+);", open(FFI).read())}
    assert consts and consts == rs


@pytest.mark.parametrize("path", [AMD])
def test_shim_calls_declared_functions_with_their_arity(path):
    decl = ffi_functions()
    src = open(path).read()
    calls = 0
    for m in re.finditer(r"ffi::(ecg_\w+)\(", src):
        name = m.group(1)
        assert name in decl, name
        depth, i = 1, m.end()
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        assert len(_split_args(src[m.end():i - 1])) == len(decl[name][1]), name
        calls += 1
    assert calls >= 15


def test_shim_mirrors_reference_entry_points():
    src = open(AMD).read()
    for sym in ("pub struct FftKernel", "pub fn radix_fft_many", "pub struct MultiexpKernel",
                "pub fn parallel_multiexp<'s>", "scope: &Scope<'s>", "pub fn multiexp(&mut self, pool: &Worker",
                "pub fn num_kernels", "pub struct SingleMultiexpKernel", "pub struct EcFftKernel",
                "pub fn radix_ec_fft_many", "pub fn upload_multiexp_bases", "pub fn multiple_multiexp",
                "\"No working GPUs found!\"", "\"Expected more bases from source.\"", "EcError::Aborted"):
        assert sym in src, sym
