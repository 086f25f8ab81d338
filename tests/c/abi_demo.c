/* Plain-C caller of libecgpu.so through include/ecgpu.h only -- the shape of
 * the FFI a Rust/Go/C prover binds.  Built by
 * tests/test_c_abi.py with gcc against the in-tree library.
 *
 *   abi_demo                 : version, runtime, device count; with no GPU,
 *                              checks the "No working GPUs found!" path
 *   abi_demo IN OUT          : IN = u64 [log_n, n_msm, omega[4],
 *                              fft data[2^log_n][4], bases[n_msm][12],
 *                              scalars[n_msm][4]]; runs ecg_fft (BLS12-381 Fr)
 *                              and ecg_msm (BLS12-381 G1) on device 0 and
 *                              writes OUT = u64 [fft out[2^log_n][4],
 *                              msm out[18]]. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ecgpu.h"

static int fail(const char *what, int rc) {
  fprintf(stderr, "%s failed: rc=%d %s\n", what, rc, ecg_last_error());
  return 1;
}

int main(int argc, char **argv) {
  printf("version: %s\nruntime: %s\n", ecg_version(), ecg_runtime_info());
  int ndev = ecg_device_count();
  printf("devices: %d\n", ndev);
  if (argc < 3) {
    if (ndev == 0) {
      ecg_ctx *ctx = NULL;
      int rc = ecg_ctx_create(0, &ctx);
      if (rc != ECG_ERR_NODEV || strstr(ecg_last_error(), "No working GPUs found!") == NULL) {
        fprintf(stderr, "expected ECG_ERR_NODEV, got %d (%s)\n", rc, ecg_last_error());
        return 1;
      }
      printf("no-device path ok\n");
    }
    return 0;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) return fail("open input", -1);
  uint64_t hdr[2];
  if (fread(hdr, 8, 2, f) != 2) return fail("read header", -1);
  const uint32_t log_n = (uint32_t)hdr[0];
  const size_t n = (size_t)1 << log_n, m = (size_t)hdr[1];
  uint64_t omega[4];
  uint64_t *data = malloc(n * 32), *bases = malloc(m * 96 + 8), *scalars = malloc(m * 32 + 8);
  uint64_t out_msm[18];
  if (fread(omega, 8, 4, f) != 4 || fread(data, 32, n, f) != n || fread(bases, 96, m, f) != m ||
      fread(scalars, 32, m, f) != m)
    return fail("read input", -1);
  fclose(f);
  ecg_ctx *ctx = NULL;
  int rc = ecg_ctx_create(0, &ctx);
  if (rc) return fail("ecg_ctx_create", rc);
  if ((rc = ecg_fft(ctx, ECG_FIELD_BLS12_381_FR, data, omega, log_n, NULL, NULL))) return fail("ecg_fft", rc);
  if ((rc = ecg_msm(ctx, ECG_CURVE_BLS12_381, bases, scalars, m, out_msm, NULL, NULL))) return fail("ecg_msm", rc);
  ecg_ctx_destroy(ctx);
  f = fopen(argv[2], "wb");
  if (!f || fwrite(data, 32, n, f) != n || fwrite(out_msm, 8, 18, f) != 18) return fail("write output", -1);
  fclose(f);
  free(data);
  free(bases);
  free(scalars);
  printf("fft 2^%u and msm of %zu terms done\n", log_n, m);
  return 0;
}
