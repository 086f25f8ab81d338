// Kernel registry and device queries of the C ABI (include/ecgpu.h).
//
// The reference generates its CUDA/OpenCL source per downstream crate at build
// time (ag_build::SourceBuilder, ag-build/src/source/builder.rs:35-152, and
// ag_build::generate, ag-build/src/lib.rs:47-53) and loads it per device
// (ec_gpu_program::program!, ec-gpu-program/src/program.rs:11-29).  Here every
// kernel is compiled into libecgpu.so ahead of time, so both steps reduce to
// asking which field / curve instantiations the library holds.  Instantiations
// are named by their moduli -- the values ag_types::GpuField::modulus() and
// ark_ff::Field::characteristic() report -- so the Rust binding resolves an id
// from any generic `F: Field` / `G: GpuCurveAffine` without a new trait bound.
#include <hip/hip_runtime.h>

#include <cstring>

#include "ctx.hpp"

namespace ecg {
namespace reg {
namespace params {
#include "params.inc"
}

struct FieldRow {
  int id;
  const char* name;
  const uint64_t* p;  // prime modulus limbs
  int n;              // limbs
  uint32_t degree;    // extension degree over the prime field
  bool fft;           // a radix-FFT field (two-adic Fr)
};

static const FieldRow kFields[] = {
    {ECG_FIELD_BLS12_381_FR, "bls12_381_fr", params::bls12_381_fr::P, 4, 1, true},
    {ECG_FIELD_BLS12_381_FQ, "bls12_381_fq", params::bls12_381_fq::P, 6, 1, false},
    {ECG_FIELD_BN254_FR, "bn254_fr", params::bn254_fr::P, 4, 1, true},
    {ECG_FIELD_BN254_FQ, "bn254_fq", params::bn254_fq::P, 4, 1, false},
    {ECG_FIELD_BLS12_381_FQ2, "bls12_381_fq2", params::bls12_381_fq::P, 6, 2, false},
    {ECG_FIELD_BN254_FQ2, "bn254_fq2", params::bn254_fq::P, 4, 2, false},
};

struct CurveRow {
  int id;
  const char* name;
  int base_field;    // coordinate field (Fq or Fq2)
  int scalar_field;  // Fr
};

static const CurveRow kCurves[] = {
    {ECG_CURVE_BLS12_381, "bls12_381_g1", ECG_FIELD_BLS12_381_FQ, ECG_FIELD_BLS12_381_FR},
    {ECG_CURVE_BN254, "bn254_g1", ECG_FIELD_BN254_FQ, ECG_FIELD_BN254_FR},
    {ECG_CURVE_BLS12_381_G2, "bls12_381_g2", ECG_FIELD_BLS12_381_FQ2, ECG_FIELD_BLS12_381_FR},
    {ECG_CURVE_BN254_G2, "bn254_g2", ECG_FIELD_BN254_FQ2, ECG_FIELD_BN254_FR},
};

static const FieldRow* field_row(int id) {
  for (const auto& f : kFields)
    if (f.id == id) return &f;
  return nullptr;
}

// limbs equal up to high zero limbs on either side
static bool same_modulus(const uint64_t* a, size_t na, const uint64_t* b, size_t nb) {
  size_t n = na > nb ? na : nb;
  for (size_t i = 0; i < n; ++i) {
    uint64_t x = i < na ? a[i] : 0, y = i < nb ? b[i] : 0;
    if (x != y) return false;
  }
  return true;
}

static int find_field(const uint64_t* m, size_t limbs, uint32_t degree) {
  for (const auto& f : kFields)
    if (f.degree == degree && same_modulus(m, limbs, f.p, f.n)) return f.id;
  return -1;
}

static void modulus_hex(const uint64_t* m, size_t limbs, char* out, size_t cap) {
  size_t k = 0;
  out[0] = 0;
  k += snprintf(out + k, cap - k, "0x");
  bool lead = true;
  for (size_t i = limbs; i-- > 0 && k + 17 < cap;) {
    if (lead && m[i] == 0 && i > 0) continue;
    k += snprintf(out + k, cap - k, lead ? "%llx" : "%016llx", (unsigned long long)m[i]);
    lead = false;
  }
}

}  // namespace reg
}  // namespace ecg

using namespace ecg;
using namespace ecg::reg;

extern "C" {

int ecg_device_info(int device, size_t* mem_bytes, int* compute_units, char* name, size_t name_cap) {
  int n = ecg_device_count();
  if (device < 0 || device >= n) {
    set_error("ecg_device_info: device %d out of range [0, %d)", device, n);
    return n <= 0 ? ECG_ERR_NODEV : ECG_ERR_INVALID;
  }
  hipDeviceProp_t prop;
  ECG_HIP(hipGetDeviceProperties(&prop, device));
  if (mem_bytes) *mem_bytes = prop.totalGlobalMem;
  if (compute_units) *compute_units = prop.multiProcessorCount;
  if (name && name_cap) snprintf(name, name_cap, "%s (%s)", prop.name, prop.gcnArchName);
  return ECG_OK;
}

int ecg_field_id(const uint64_t* modulus, size_t limbs, uint32_t degree) {
  if (!modulus || limbs == 0) {
    set_error("ecg_field_id: empty modulus");
    return ECG_ERR_INVALID;
  }
  int id = find_field(modulus, limbs, degree);
  if (id < 0) {
    char hex[200];
    modulus_hex(modulus, limbs, hex, sizeof hex);
    set_error("libecgpu.so has no kernels for the degree-%u field over modulus %s", degree, hex);
    return ECG_ERR_INVALID;
  }
  return id;
}

int ecg_curve_id(const uint64_t* base_modulus, size_t base_limbs, uint32_t base_degree,
                 const uint64_t* scalar_modulus, size_t scalar_limbs) {
  if (!base_modulus || !scalar_modulus || !base_limbs || !scalar_limbs) {
    set_error("ecg_curve_id: empty modulus");
    return ECG_ERR_INVALID;
  }
  int fb = find_field(base_modulus, base_limbs, base_degree);
  int fs = find_field(scalar_modulus, scalar_limbs, 1);
  for (const auto& c : kCurves)
    if (c.base_field == fb && c.scalar_field == fs) return c.id;
  char hb[200], hs[200];
  modulus_hex(base_modulus, base_limbs, hb, sizeof hb);
  modulus_hex(scalar_modulus, scalar_limbs, hs, sizeof hs);
  set_error("libecgpu.so has no curve over the degree-%u field of %s with scalars mod %s", base_degree, hb, hs);
  return ECG_ERR_INVALID;
}

int ecg_has_kernel(int kind, int id) {
  switch (kind) {
    case ECG_KIND_FIELD:
      return field_row(id) != nullptr;
    case ECG_KIND_FFT: {
      const FieldRow* f = field_row(id);
      return f && f->fft;
    }
    case ECG_KIND_EC:
    case ECG_KIND_EC_FFT:
    case ECG_KIND_MULTIEXP:
      for (const auto& c : kCurves)
        if (c.id == id) return 1;
      return 0;
    default:
      return 0;
  }
}

const char* ecg_field_name(int field_id) {
  const FieldRow* f = field_row(field_id);
  return f ? f->name : nullptr;
}

const char* ecg_curve_name(int curve_id) {
  for (const auto& c : kCurves)
    if (c.id == curve_id) return c.name;
  return nullptr;
}

}  // extern "C"
