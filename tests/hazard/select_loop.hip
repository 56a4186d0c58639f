// GPU side of the selection-loop hazard check (see select_loop.h): one thread per run computes the
// three digests; the host computes the same on the CPU and counts the runs where they differ.
// Build: make -C tests/hazard   Run: ./select_loop [runs]   (prints mismatches per form)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "select_loop.h"

constexpr uint32_t kMaxLen = 12;

__global__ void __launch_bounds__(256) digests(uint32_t nruns, uint64_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < nruns;
  SlRow rows[kMaxLen];
  const uint32_t n = act ? sl_len(i) : 0;
  for (uint32_t k = 0; k < kMaxLen; ++k) rows[k] = sl_row(i, k);
  uint32_t kmax = n;
  for (int o = 32; o > 0; o >>= 1) kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o, 64));
  const uint64_t a = act ? sl_divergent_if(rows, n) : 0;
  const uint64_t b = act ? sl_divergent_select(rows, n) : 0;
  const uint64_t c = sl_uniform(rows, n, kmax);
  if (act) {
    out[3 * (uint64_t)i] = a;
    out[3 * (uint64_t)i + 1] = b;
    out[3 * (uint64_t)i + 2] = c;
  }
}

int main(int argc, char** argv) {
  const uint32_t nruns = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : (1u << 20);
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 24ull * nruns) != hipSuccess) return 2;
  digests<<<(nruns + 255) / 256, 256>>>(nruns, d);
  std::vector<uint64_t> h(3ull * nruns);
  if (hipMemcpy(h.data(), d, 24ull * nruns, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  (void)hipFree(d);
  uint64_t bad[3] = {0, 0, 0};
  for (uint32_t i = 0; i < nruns; ++i) {
    SlRow rows[kMaxLen];
    for (uint32_t k = 0; k < kMaxLen; ++k) rows[k] = sl_row(i, k);
    const uint32_t n = sl_len(i);
    const uint64_t want = sl_divergent_if(rows, n);  // the three forms agree on the CPU (select_loop_host)
    bad[0] += h[3ull * i] != want;
    bad[1] += h[3ull * i + 1] != want;
    bad[2] += h[3ull * i + 2] != want;
  }
  printf("{\"runs\": %u, \"mismatch_divergent_if\": %llu, \"mismatch_divergent_select\": %llu, \"mismatch_uniform\": %llu}\n",
         nruns, (unsigned long long)bad[0], (unsigned long long)bad[1], (unsigned long long)bad[2]);
  return 0;
}
