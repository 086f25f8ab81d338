// Sort microbenchmark for the MSM's per-window bucket sort (dev tool).
// One window block of the 2^26 MSM: N (key, value) pairs, keys uniform in
// [0, 2^19) (|digit| - 1 at c = 20) plus the block sentinel bit 19, values
// 32-bit term indices.  Times rocPRIM onesweep configurations for 20-bit
// keys, and the keys-only u64 form (key << 32 | value, bits [32, 52)).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o sort_bench sort_bench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rocprim/rocprim.hpp>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

template <int BS, int IPT, int BITS, rocprim::block_radix_rank_algorithm ALG>
using Cfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>, rocprim::kernel_config<BS, IPT>, BITS, ALG>>;

__global__ void gen(uint32_t* k, uint32_t* v, uint64_t* kv, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  uint32_t key = x & ((1u << 19) - 1);
  if ((x >> 19) == 0) key |= 1u << 19;  // rare sentinel
  k[i] = key;
  v[i] = (uint32_t)i | ((x >> 31) << 31);
  kv[i] = ((uint64_t)key << 32) | v[i];
}

__global__ void check_pairs(const uint32_t* k, size_t n, unsigned* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 < n && k[i] > k[i + 1]) atomicAdd(bad, 1u);
}
__global__ void check_kv(const uint64_t* k, size_t n, unsigned* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 < n && (k[i] >> 32) > (k[i + 1] >> 32)) atomicAdd(bad, 1u);
}

// 6-byte entries: 20-bit key in the low bits (w[0] + low 4 bits of w[1]),
// 28 value bits above -- 6 B instead of 8 B moved per entry and pass.
struct K6 {
  uint16_t w[3];
};
struct K6Dec {
  __host__ __device__ rocprim::tuple<uint16_t&, uint16_t&, uint16_t&> operator()(K6& k) const {
    return rocprim::tuple<uint16_t&, uint16_t&, uint16_t&>(k.w[2], k.w[1], k.w[0]);
  }
};
__global__ void gen6(const uint64_t* kv, K6* k6, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t key = (uint32_t)(kv[i] >> 32), val = (uint32_t)kv[i] & 0x0fffffffu;
  K6 e;
  e.w[0] = (uint16_t)key;
  e.w[1] = (uint16_t)((key >> 16) | ((val & 0xfffu) << 4));
  e.w[2] = (uint16_t)(val >> 12);
  k6[i] = e;
}
__global__ void check_k6(const K6* k, size_t n, unsigned* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i + 1 >= n) return;
  const uint32_t a = k[i].w[0] | ((uint32_t)(k[i].w[1] & 15) << 16);
  const uint32_t b = k[i + 1].w[0] | ((uint32_t)(k[i + 1].w[1] & 15) << 16);
  if (a > b) atomicAdd(bad, 1u);
}

struct Bufs {
  uint32_t *k0, *k1, *v0, *v1;
  uint64_t *kv0, *kv1;
  void* tmp;
  size_t tmp_bytes;
  unsigned* bad;
  size_t n;
};

template <class C>
void run_pairs(const char* name, Bufs& b, hipStream_t s) {
  size_t bytes = 0;
  CHK(rocprim::radix_sort_pairs<C>(nullptr, bytes, b.k0, b.k1, b.v0, b.v1, b.n, 0, 20, s));
  if (bytes > b.tmp_bytes) { printf("%-40s tmp %zu too big\n", name, bytes); return; }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e9, sum = 0;
  const int reps = 7;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(e0, s));
    CHK(rocprim::radix_sort_pairs<C>(b.tmp, bytes, b.k0, b.k1, b.v0, b.v1, b.n, 0, 20, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) { best = ms < best ? ms : best; sum += ms; }
  }
  CHK(hipMemsetAsync(b.bad, 0, 4, s));
  check_pairs<<<(b.n + 255) / 256, 256, 0, s>>>(b.k1, b.n, b.bad);
  unsigned bad; CHK(hipMemcpy(&bad, b.bad, 4, hipMemcpyDeviceToHost));
  const double gb = 2.0 * 16.0 * b.n / 1e9 + 4.0 * b.n / 1e9;  // 2 passes x (8 B in + 8 B out) + histogram
  printf("%-40s best %.3f ms avg %.3f ms  %.2f TB/s (36 B/pair)  %s\n", name, best, sum / (reps - 1),
         gb / best, bad ? "UNSORTED" : "ok");
}

template <class C>
void run_kv(const char* name, Bufs& b, hipStream_t s) {
  size_t bytes = 0;
  CHK(rocprim::radix_sort_keys<C>(nullptr, bytes, b.kv0, b.kv1, b.n, 32, 52, s));
  if (bytes > b.tmp_bytes) { printf("%-40s tmp %zu too big\n", name, bytes); return; }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e9, sum = 0;
  const int reps = 7;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(e0, s));
    CHK(rocprim::radix_sort_keys<C>(b.tmp, bytes, b.kv0, b.kv1, b.n, 32, 52, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) { best = ms < best ? ms : best; sum += ms; }
  }
  CHK(hipMemsetAsync(b.bad, 0, 4, s));
  check_kv<<<(b.n + 255) / 256, 256, 0, s>>>(b.kv1, b.n, b.bad);
  unsigned bad; CHK(hipMemcpy(&bad, b.bad, 4, hipMemcpyDeviceToHost));
  const double gb = 2.0 * 16.0 * b.n / 1e9 + 8.0 * b.n / 1e9;
  printf("%-40s best %.3f ms avg %.3f ms  %.2f TB/s  %s\n", name, best, sum / (reps - 1), gb / best, bad ? "UNSORTED" : "ok");
}

template <class C>
void run_k6(const char* name, Bufs& b, K6* a, K6* o, hipStream_t s) {
  size_t bytes = 0;
  CHK(rocprim::radix_sort_keys<C>(nullptr, bytes, a, o, b.n, K6Dec{}, 0, 20, s));
  if (bytes > b.tmp_bytes) { printf("%-40s tmp %zu too big\n", name, bytes); return; }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  float best = 1e9, sum = 0;
  const int reps = 7;
  for (int r = 0; r < reps; r++) {
    CHK(hipEventRecord(e0, s));
    CHK(rocprim::radix_sort_keys<C>(b.tmp, bytes, a, o, b.n, K6Dec{}, 0, 20, s));
    CHK(hipEventRecord(e1, s));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) { best = ms < best ? ms : best; sum += ms; }
  }
  CHK(hipMemsetAsync(b.bad, 0, 4, s));
  check_k6<<<(b.n + 255) / 256, 256, 0, s>>>(o, b.n, b.bad);
  unsigned bad; CHK(hipMemcpy(&bad, b.bad, 4, hipMemcpyDeviceToHost));
  const double gb = 2.0 * 12.0 * b.n / 1e9 + 6.0 * b.n / 1e9;
  printf("%-40s best %.3f ms avg %.3f ms  %.2f TB/s  %s\n", name, best, sum / (reps - 1), gb / best, bad ? "UNSORTED" : "ok");
}

int main(int argc, char** argv) {
  const int logn = argc > 1 ? atoi(argv[1]) : 26;
  Bufs b;
  b.n = (size_t)1 << logn;
  CHK(hipMalloc(&b.k0, b.n * 4)); CHK(hipMalloc(&b.k1, b.n * 4));
  CHK(hipMalloc(&b.v0, b.n * 4)); CHK(hipMalloc(&b.v1, b.n * 4));
  CHK(hipMalloc(&b.kv0, b.n * 8)); CHK(hipMalloc(&b.kv1, b.n * 8));
  b.tmp_bytes = (size_t)1 << 30;
  CHK(hipMalloc(&b.tmp, b.tmp_bytes));
  CHK(hipMalloc(&b.bad, 4));
  hipStream_t s;
  CHK(hipStreamCreate(&s));
  gen<<<(b.n + 255) / 256, 256, 0, s>>>(b.k0, b.v0, b.kv0, b.n, 12345);
  CHK(hipStreamSynchronize(s));
  using A = rocprim::block_radix_rank_algorithm;
  printf("n = 2^%d pairs (20-bit keys)\n", logn);
  run_pairs<rocprim::default_config>("pairs default", b, s);
  run_pairs<Cfg<1024, 8, 10, A::match>>("pairs 1024x8 r10 match", b, s);
  run_pairs<Cfg<1024, 12, 10, A::match>>("pairs 1024x12 r10 match (current)", b, s);
  run_pairs<Cfg<512, 16, 10, A::match>>("pairs 512x16 r10 match", b, s);
  run_pairs<Cfg<512, 24, 10, A::match>>("pairs 512x24 r10 match", b, s);
  run_pairs<Cfg<256, 24, 10, A::match>>("pairs 256x24 r10 match", b, s);
  run_pairs<Cfg<1024, 16, 10, A::match>>("pairs 1024x16 r10 match", b, s);
  run_pairs<Cfg<1024, 12, 11, A::match>>("pairs 1024x12 r11 match", b, s);
  run_pairs<Cfg<1024, 12, 8, A::match>>("pairs 1024x12 r8 match (3 passes)", b, s);
  if (argc > 2) {  // 6-byte entries only (plus the current u64 form for reference)
    K6 *a6, *o6;
    CHK(hipMalloc(&a6, b.n * 6)); CHK(hipMalloc(&o6, b.n * 6));
    gen6<<<(b.n + 255) / 256, 256, 0, s>>>(b.kv0, a6, b.n);
    CHK(hipStreamSynchronize(s));
    run_kv<Cfg<1024, 12, 10, A::match>>("u64 keys 1024x12 r10 match (current)", b, s);
    run_k6<Cfg<1024, 12, 10, A::match>>("K6 keys 1024x12 r10 match", b, a6, o6, s);
    run_k6<Cfg<1024, 16, 10, A::match>>("K6 keys 1024x16 r10 match", b, a6, o6, s);
    run_k6<Cfg<1024, 8, 10, A::match>>("K6 keys 1024x8 r10 match", b, a6, o6, s);
    run_k6<Cfg<512, 16, 10, A::match>>("K6 keys 512x16 r10 match", b, a6, o6, s);
    run_k6<rocprim::default_config>("K6 keys default", b, a6, o6, s);
    return 0;
  }
  run_kv<Cfg<1024, 12, 10, A::match>>("u64 keys 1024x12 r10 match", b, s);
  run_kv<Cfg<512, 16, 10, A::match>>("u64 keys 512x16 r10 match", b, s);
  run_kv<Cfg<1024, 8, 10, A::match>>("u64 keys 1024x8 r10 match", b, s);
  return 0;
}
