// Device-scope atomic contention probe: 256 workgroups x 8 waves (the re-score launch's grid),
// lane 0 of every wave does K dependent fetch-adds (agent scope, relaxed -- the re-score claim's
// atomic) on counter[wave_id % NC].  Kernel time vs NC shows whether one shared cursor
// serialises the claims of a burst tick (ewk_rescore.h rs_claim).
//   hipcc --offload-arch=gfx950 -O3 scripts/probes/atomic_probe.hip -o scripts/probes/atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(512) void k_claims(int* ctr, int nc, int k, int* sink) {
    const int wave = blockIdx.x * 8 + (threadIdx.x >> 6);
    int acc = 0;
    if ((threadIdx.x & 63) == 0) {
        int* p = ctr + 64 * (wave % nc);   // one counter per 256-B line
        for (int i = 0; i < k; ++i) {
            const int g = __hip_atomic_fetch_add(p, 1 + (acc & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += g;   // the next claim depends on this one (as a wave's claims do)
        }
        if (acc == -1) sink[wave] = acc;
    }
}

int main() {
    int *ctr, *sink;
    hipMalloc(&ctr, 64 * 64 * sizeof(int) * 64);
    hipMalloc(&sink, 2048 * sizeof(int));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int ncs[] = {1, 8, 64, 2048};
    const int ks[] = {0, 1, 4, 16};
    for (int nc : ncs) {
        for (int k : ks) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipMemset(ctr, 0, 64 * 64 * sizeof(int) * 64);
                hipEventRecord(a);
                hipLaunchKernelGGL(k_claims, dim3(256), dim3(512), 0, 0, ctr, nc, k, sink);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            printf("counters %4d  claims per wave %2d  kernel %8.2f us  (%d atomics)\n", nc, k, best * 1e3f, 2048 * k);
        }
    }
    return 0;
}
