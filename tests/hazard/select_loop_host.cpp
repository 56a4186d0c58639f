// Host side of the selection-loop hazard check (see select_loop.h): the three forms on the CPU,
// built under -fsanitize=undefined (and memory with clang): any undefined behaviour in the loop
// source (an uninitialised loop-carried row read on a zero-trip lane, say) is reported here.
// Prints the number of runs where the forms disagree (0 expected) and exits 1 otherwise.
#include <stdio.h>
#include <stdlib.h>

#include "select_loop.h"

int main(int argc, char** argv) {
  const uint32_t nruns = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : 200000;
  uint64_t disagree = 0;
  for (uint32_t i = 0; i < nruns; ++i) {
    SlRow rows[12];
    for (uint32_t k = 0; k < 12; ++k) rows[k] = sl_row(i, k);
    const uint32_t n = sl_len(i);
    const uint64_t a = sl_divergent_if(rows, n), b = sl_divergent_select(rows, n);
    // the uniform form with the trip count of a wave whose largest run is 12, and of this run alone
    const uint64_t c = sl_uniform(rows, n, 12), d = sl_uniform(rows, n, n);
    disagree += (a != b) || (a != c) || (a != d);
  }
  printf("{\"runs\": %u, \"forms_disagree\": %llu}\n", nruns, (unsigned long long)disagree);
  return disagree ? 1 : 0;
}
