// curve_id -> curve type dispatch for the host drivers (G1 and G2 of both
// curves; ids in include/ecgpu.h).
#pragma once
#include <type_traits>

#include "ctx.hpp"
#include "curve.hpp"
#include "host_field.hpp"

namespace ecg {

// Host coordinate field matching a curve's device Fq (HFp for G1, HFp2 for G2).
template <class C>
using HostF = std::conditional_t<C::EXT == 1, host::HFp<typename C::FqParams>, host::HFp2<typename C::FqParams>>;

// Calls f(C{}) with the curve type of curve_id.
template <class Fn>
static int with_curve(int curve_id, const char* what, Fn&& f) {
  switch (curve_id) {
    case ECG_CURVE_BLS12_381: return f(BLS12_381{});
    case ECG_CURVE_BN254: return f(BN254{});
    case ECG_CURVE_BLS12_381_G2: return f(BLS12_381_G2{});
    case ECG_CURVE_BN254_G2: return f(BN254_G2{});
    default:
      set_error("%s: unknown curve_id %d", what, curve_id);
      return ECG_ERR_INVALID;
  }
}

}  // namespace ecg
