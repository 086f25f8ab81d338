// Element-wise field operations on the device (ecg_field_ops): the reference's
// GPU field tests (ag-build/src/tests/test_fields.rs: test_add / test_sub /
// test_mul / test_pow / test_sqr / test_double / test_mont / test_unmont,
// which run one field.cl function per kernel, field.cl:14-392) restated over
// the engine's field forms, so each form's arithmetic is checked on its own
// and not only through the MSM / NTT results:
//   form 0: the boundary form (field.hpp: 32-bit limbs, R = 2^(64N), fully
//           reduced) -- EC-FFT stages, G2, every boundary conversion;
//   form 1: the reduced-radix form of the product path (fieldrr.hpp) -- MSM
//           buckets (BLS12-381 Fq 13 x 30, BN254 Fq 9 x 29) and the NTT
//           (Fr 9 x 29);
//   form 2: the second reduced-radix form of an Fq (BLS12-381 Fq 14 x 29,
//           BN254 Fq 10 x 28: the G2 MSM's Fq2 components).
// Reduced-radix operands enter through rr_from_std and leave through
// rr_to_std (canonical), so every form returns the same bytes.
#include <cstring>

#include "ctx.hpp"
#include "fieldrr.hpp"

namespace ecg {

template <class P>
ECG_DEV Fp<P> bnd_op(int op, const Fp<P>& x, const Fp<P>& y, uint32_t e) {
  switch (op) {
    case ECG_FOP_ADD: return fadd(x, y);
    case ECG_FOP_SUB: return fsub(x, y);
    case ECG_FOP_MUL: return fmul(x, y);
    case ECG_FOP_SQR: return fsqr(x);
    case ECG_FOP_DOUBLE: return fdbl(x);
    case ECG_FOP_POW: return fpow_u32(x, e);
    case ECG_FOP_MONT: return to_mont(x);
    case ECG_FOP_UNMONT: return from_mont(x);
    case ECG_FOP_INV: return finv(x);
    default: return x;
  }
}

// a^e in the reduced-radix form (square-and-multiply, LSB first; product
// outputs stay below 1.5 p, inside every product's operand bound)
template <class Q>
ECG_DEV FpR<Q> rr_pow_u32(FpR<Q> base, uint32_t e) {
  FpR<Q> r = FpR<Q>::one();
  while (e) {
    if (e & 1) r = rr_mul(r, base);
    e >>= 1;
    if (e) base = rr_sqr(base);
  }
  return r;
}

template <class Q>
ECG_DEV FpR<Q> rr_inv_fermat(const FpR<Q>& a) {  // a^(p-2), MSB first
  using P = typename Q::Base;
  FpR<Q> r = FpR<Q>::one();
  for (int i = P::N - 1; i >= 0; i--) {
    const uint64_t e = P::PM2[i];
    for (int bit = 63; bit >= 0; bit--) {
      r = rr_sqr(r);
      if ((e >> bit) & 1) r = rr_mul(r, a);
    }
  }
  return r;
}

template <class Q>
ECG_DEV Fp<typename Q::Base> rr_op(int op, const Fp<typename Q::Base>& x, const Fp<typename Q::Base>& y, uint32_t e) {
  const FpR<Q> u = rr_from_std<Q>(x), w = rr_from_std<Q>(y);
  switch (op) {
    case ECG_FOP_ADD: return rr_to_std(rr_add(u, w));
    case ECG_FOP_SUB: return rr_to_std(rr_sub<4>(u, w));  // w < 1.5 p <= 4p / 2
    case ECG_FOP_MUL: return rr_to_std(rr_mul(u, w));
    case ECG_FOP_SQR: return rr_to_std(rr_sqr(u));
    case ECG_FOP_DOUBLE: return rr_to_std(rr_add(u, u));
    case ECG_FOP_POW: return rr_to_std(rr_pow_u32(u, e));
    case ECG_FOP_INV: return rr_to_std(rr_inv_fermat(u));
    default: return rr_to_std(u);  // the radix change both ways
  }
}

template <class P, class Q1, class Q2>
__global__ void field_ops_kernel(int form, int op, const Fp<P>* __restrict__ a, const Fp<P>* __restrict__ b,
                                 uint32_t e, size_t n, Fp<P>* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fp<P> x = load(&a[i]), y = load(&b[i]);
  Fp<P> r;
  if (form == 0)
    r = bnd_op(op, x, y, e);
  else if (form == 1)
    r = rr_op<Q1>(op, x, y, e);
  else
    r = rr_op<Q2>(op, x, y, e);
  store(&out[i], r);
}

template <class P, class Q1, class Q2>
static int field_ops_t(ecg_ctx* ctx, int form, int op, const uint64_t* a, const uint64_t* b, uint32_t e, size_t n,
                       uint64_t* out, hipStream_t s) {
  using F = Fp<P>;
  void *da, *db, *dout;
  ECG_TRY(ws_get(ctx, "fops_a", n * sizeof(F), &da));
  ECG_TRY(ws_get(ctx, "fops_b", n * sizeof(F), &db));
  ECG_TRY(ws_get(ctx, "fops_out", n * sizeof(F), &dout));
  ECG_HIP(hipMemcpyAsync(da, a, n * sizeof(F), hipMemcpyHostToDevice, s));
  if (b)
    ECG_HIP(hipMemcpyAsync(db, b, n * sizeof(F), hipMemcpyHostToDevice, s));
  else
    ECG_HIP(hipMemsetAsync(db, 0, n * sizeof(F), s));
  hipLaunchKernelGGL((field_ops_kernel<P, Q1, Q2>), dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, s, form, op,
                     (const F*)da, (const F*)db, e, n, (F*)dout);
  ECG_HIP(hipGetLastError());
  ECG_HIP(hipMemcpyAsync(out, dout, n * sizeof(F), hipMemcpyDeviceToHost, s));
  ECG_HIP(hipStreamSynchronize(s));
  return ECG_OK;
}

}  // namespace ecg

using namespace ecg;

extern "C" int ecg_field_ops(ecg_ctx* ctx, int field_id, int form, int op, const uint64_t* a, const uint64_t* b,
                             uint32_t e, size_t n, uint64_t* out) {
  ECG_ENTER(ctx);
  if (!a || !out || ((op == ECG_FOP_ADD || op == ECG_FOP_SUB || op == ECG_FOP_MUL) && !b)) {
    set_error("field_ops: null pointer");
    return ECG_ERR_INVALID;
  }
  if (op < ECG_FOP_ADD || op > ECG_FOP_INV || form < 0 || form > 2 ||
      (form > 0 && (op == ECG_FOP_MONT || op == ECG_FOP_UNMONT))) {
    set_error("field_ops: op %d / form %d not supported (forms 1-2 take values in Montgomery form and have no "
              "mont / unmont)", op, form);
    return ECG_ERR_INVALID;
  }
  const bool fr = field_id == ECG_FIELD_BLS12_381_FR || field_id == ECG_FIELD_BN254_FR;
  if (form == 2 && fr) {
    set_error("field_ops: form 2 exists for the base fields (Fq) only");
    return ECG_ERR_INVALID;
  }
  if (n == 0) return ECG_OK;
  hipStream_t s = ctx->stream;
  switch (field_id) {
    case ECG_FIELD_BLS12_381_FR:
      return field_ops_t<params::bls12_381_fr, params::bls12_381_fr_rr, params::bls12_381_fr_rr>(ctx, form, op, a, b,
                                                                                                  e, n, out, s);
    case ECG_FIELD_BLS12_381_FQ:
      return field_ops_t<params::bls12_381_fq, params::bls12_381_fq13_rr, params::bls12_381_fq_rr>(ctx, form, op, a,
                                                                                                    b, e, n, out, s);
    case ECG_FIELD_BN254_FR:
      return field_ops_t<params::bn254_fr, params::bn254_fr_rr, params::bn254_fr_rr>(ctx, form, op, a, b, e, n, out,
                                                                                      s);
    case ECG_FIELD_BN254_FQ:
      return field_ops_t<params::bn254_fq, params::bn254_fq9_rr, params::bn254_fq_rr>(ctx, form, op, a, b, e, n, out,
                                                                                       s);
    default:
      set_error("field_ops: unknown field_id %d", field_id);
      return ECG_ERR_INVALID;
  }
}
