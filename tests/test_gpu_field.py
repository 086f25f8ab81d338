"""The engine's field arithmetic on the GPU, operation by operation -- the
reference's own GPU field tests (ag-build/src/tests/test_fields.rs: test_add,
test_sub, test_mul, test_pow, test_sqr, test_double, test_mont, test_unmont,
each running one field.cl function on random elements against arkworks),
restated over every field form the engine computes in (ecg_field_ops):
form 0 the boundary form (field.hpp), form 1 the product path's reduced-radix
form (Fr 9 x 29, BLS12-381 Fq 13 x 30, BN254 Fq 9 x 29), form 2 an Fq's G2
reduced-radix form (14 x 29, 10 x 28).  Expected values come from Python
integers (py_oracle's field constants); results must be equal byte for byte
(canonical Montgomery)."""
import numpy as np
import pytest

import coracle as co
import ecgpu
import py_oracle as po

pytestmark = pytest.mark.gpu

CASES = [("bls12_381_fr", 0), ("bls12_381_fr", 1), ("bls12_381_fq", 0), ("bls12_381_fq", 1), ("bls12_381_fq", 2),
         ("bn254_fr", 0), ("bn254_fr", 1), ("bn254_fq", 0), ("bn254_fq", 1), ("bn254_fq", 2)]


def _elems(f, n, seed):
    """n Montgomery representatives: random canonical values plus the edges 0, 1, p - 1, 2."""
    rng = po.Xoshiro256ss(seed)
    xs = [0, 1, f.modulus - 1, 2] + [rng.field_element(f) for _ in range(n - 4)]
    return xs, co.u64arr([f.to_mont(x) for x in xs], (f.modulus.bit_length() + 63) // 64)


@pytest.mark.parametrize("fname,form", CASES)
def test_field_ops_match_integers(gpu_programs, fname, form):
    prog = gpu_programs[0][0]
    f = po.FIELDS[fname]
    p = f.modulus
    n = 256
    xs, A = _elems(f, n, 11 + form)
    ys, B = _elems(f, n, 29 + form)
    ys = ys[4:] + ys[:4]  # pair the edges with random values too
    B = np.ascontiguousarray(np.concatenate([B[4:], B[:4]]))
    limbs = A.shape[1]

    def mont(vals):
        return co.u64arr([f.to_mont(v % p) for v in vals], limbs)

    def run(op, b=None, e=0):
        return ecgpu.field_ops(prog, fname, form, op, A, b, e)

    assert (run(ecgpu.FOP_ADD, B) == mont([x + y for x, y in zip(xs, ys)])).all()        # test_add
    assert (run(ecgpu.FOP_SUB, B) == mont([x - y for x, y in zip(xs, ys)])).all()        # test_sub
    assert (run(ecgpu.FOP_MUL, B) == mont([x * y for x, y in zip(xs, ys)])).all()        # test_mul
    assert (run(ecgpu.FOP_SQR) == mont([x * x for x in xs])).all()                       # test_sqr
    assert (run(ecgpu.FOP_DOUBLE) == mont([2 * x for x in xs])).all()                    # test_double
    for e in (0, 1, 0xDEADBEEF):                                                         # test_pow (u32 exponent)
        assert (run(ecgpu.FOP_POW, e=e) == mont([pow(x, e, p) for x in xs])).all(), e
    inv = run(ecgpu.FOP_INV)                                                             # Fermat inverse, 0 -> 0
    assert (inv == mont([pow(x, p - 2, p) for x in xs])).all()
    if form == 0:  # test_mont / test_unmont: canonical <-> Montgomery
        canon = co.u64arr(xs, limbs)
        assert (ecgpu.field_ops(prog, fname, 0, ecgpu.FOP_MONT, canon) == A).all()
        assert (ecgpu.field_ops(prog, fname, 0, ecgpu.FOP_UNMONT, A) == canon).all()


def test_field_ops_rejects(gpu_programs):
    prog = gpu_programs[0][0]
    a = np.zeros((4, 4), np.uint64)
    with pytest.raises(ecgpu.EcError):
        ecgpu.field_ops(prog, "bls12_381_fr", 2, ecgpu.FOP_ADD, a, a)     # no second rr form for Fr
    with pytest.raises(ecgpu.EcError):
        ecgpu.field_ops(prog, "bls12_381_fr", 1, ecgpu.FOP_MONT, a)       # rr forms take Montgomery values
    with pytest.raises(ecgpu.EcError):
        ecgpu.field_ops(prog, "bls12_381_fr", 0, ecgpu.FOP_MUL, a)        # binary op without b
    with pytest.raises(ecgpu.EcError):
        ecgpu.field_ops(prog, 9, 0, ecgpu.FOP_ADD, a, a)                  # unknown field
