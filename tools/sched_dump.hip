// Prints the compile-time Poseidon2 constant schedule of csrc/poseidon2.hpp (p2::sched::V) as
// JSON, so tests/test_poseidon2_sched.py can compare it with an independent derivation.  Host
// code only (no HIP calls): runs on a CPU-only machine.
// build: hipcc -O1 -std=c++17 --offload-arch=gfx950 -o tools/sched_dump tools/sched_dump.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../era-boojum_amd/csrc/poseidon2.hpp"

static void row(const char* name, const uint64_t* v, int n, bool last = false) {
    printf("\"%s\": [", name);
    for (int i = 0; i < n; i++) printf("%s\"%llu\"", i ? ", " : "", (unsigned long long)v[i]);
    printf("]%s\n", last ? "" : ",");
}

int main() {
    constexpr p2::sched::Values v = p2::sched::V;
    printf("{\n");
    row("k", v.k, 11);
    row("d", v.d, 10);
    row("rc26", v.rc26, 12);
    printf("\"full_rc_bound\": \"%llu\", \"limb_rc_bound\": \"%llu\"\n}\n",
           (unsigned long long)p2::sched::FULL_RC_BOUND, (unsigned long long)p2::sched::LIMB_RC_BOUND);
    return 0;
}
