// Probe: is a kernel boundary (same stream) a sufficient hand-off between XCDs when the reading
// XCD's L2 already holds the lines?  (round-6 ring-path miss: could the ring scorer read ring
// lines its XCD's L2 kept from a read one ring wrap earlier, after another XCD's gate rewrote
// them?)
//   warm(r):  workgroups on XCD r read the region (plain buffer loads: lines into r's L2)
//   write(w): workgroups on XCD w rewrite it (value pattern v; non-temporal 16-B stores like the
//             gate's ring writes, or plain stores)
//   check(r): workgroups on XCD r read it back (buffer loads like the scorer) and count words
//             that are not pattern v
// Workgroups learn their XCD from HW_REG_XCC_ID and take chunks from a per-XCD counter, so the
// placement is exact whatever the dispatcher does.  Region 1 MiB (fits one XCD's 4 MiB L2).
// Build: hipcc --offload-arch=gfx950 -O3 xcd_boundary_probe.hip -o xcd_boundary_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kN = 1 << 18;          // floats (1 MiB)
constexpr int kChunk = 1024;         // floats per claim
constexpr int kChunks = kN / kChunk;

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 15;
}

__device__ __forceinline__ float pat(int v, int i) { return (float)(v * 7919 + i); }

// mode 0 warm, 1 write nt, 2 write plain, 3 check
__global__ __launch_bounds__(256) void k_step(float* buf, int* ctr, int* errs, float* sink, int mode, int xcd, int v) {
    __shared__ int chunk;
    if (xcc_id() != xcd) return;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, kN * 4, 0x00020000);
    float acc = 0.0f;
    int bad = 0;
    for (;;) {
        if (threadIdx.x == 0) chunk = atomicAdd(&ctr[xcd], 1);
        __syncthreads();
        const int c = chunk;
        __syncthreads();
        if (c >= kChunks) break;
        const int i0 = c * kChunk + 4 * threadIdx.x;   // 256 threads x 4 floats = one chunk
        if (mode == 0 || mode == 3) {
            float x[4];
            for (int k = 0; k < 4; ++k)
                x[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (i0 + k) * 4, 0, 0));
            for (int k = 0; k < 4; ++k) {
                acc += x[k];
                if (mode == 3 && x[k] != pat(v, i0 + k)) ++bad;
            }
        } else {
            typedef float f4 __attribute__((ext_vector_type(4)));
            f4 y = {pat(v, i0), pat(v, i0 + 1), pat(v, i0 + 2), pat(v, i0 + 3)};
            if (mode == 1) __builtin_nontemporal_store(y, reinterpret_cast<f4*>(buf + i0));
            else *reinterpret_cast<f4*>(buf + i0) = y;
        }
    }
    if (bad) atomicAdd(&errs[0], bad);
    if (acc == 12345.678f) sink[blockIdx.x] = acc;   // keeps the warm loads
}

__global__ void k_reset(int* ctr) { if (threadIdx.x < 16) ctr[threadIdx.x] = 0; }

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 400;
    float *buf, *sink;
    int *ctr, *errs;
    hipMalloc(&buf, kN * 4);
    hipMalloc(&sink, 4096 * 4);
    hipMalloc(&ctr, 16 * 4);
    hipMalloc(&errs, 4 * 4);
    hipMemset(buf, 0, kN * 4);
    const dim3 grid(2048), blk(256);
    const char* names[4] = {"cross-XCD, nt stores", "cross-XCD, plain stores", "same XCD, nt stores", "same XCD, plain"};
    int v = 1;
    // initial contents = pattern 0
    hipLaunchKernelGGL(k_reset, 1, 64, 0, 0, ctr);
    for (int x = 0; x < 8; ++x) {
        hipLaunchKernelGGL(k_reset, 1, 64, 0, 0, ctr);
        hipLaunchKernelGGL(k_step, grid, blk, 0, 0, buf, ctr, errs, sink, 2, x, 0);
    }
    for (int variant = 0; variant < 4; ++variant) {
        hipMemset(errs, 0, 16);
        int checked = 0;
        for (int it = 0; it < iters; ++it) {
            const int rx = it % 8;
            const int wx = variant >= 2 ? rx : (rx + 1 + (it / 8) % 7) % 8;
            const int wmode = (variant % 2 == 0) ? 1 : 2;
            hipLaunchKernelGGL(k_reset, 1, 64, 0, 0, ctr);
            hipLaunchKernelGGL(k_step, grid, blk, 0, 0, buf, ctr, errs, sink, 0, rx, v - 1);   // warm r's L2
            hipLaunchKernelGGL(k_reset, 1, 64, 0, 0, ctr);
            hipLaunchKernelGGL(k_step, grid, blk, 0, 0, buf, ctr, errs, sink, wmode, wx, v);  // rewrite on w
            hipLaunchKernelGGL(k_reset, 1, 64, 0, 0, ctr);
            hipLaunchKernelGGL(k_step, grid, blk, 0, 0, buf, ctr, errs, sink, 3, rx, v);      // check on r
            ++v;
            ++checked;
        }
        hipDeviceSynchronize();
        int e = 0;
        hipMemcpy(&e, errs, 4, hipMemcpyDeviceToHost);
        printf("%-26s %d rounds x %d words: %d stale words\n", names[variant], checked, kN, e);
        fflush(stdout);
    }
    const hipError_t err = hipGetLastError();
    printf("hip: %s\n", hipGetErrorString(err));
    return 0;
}
