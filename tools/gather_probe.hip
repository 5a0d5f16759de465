// gather_probe.hip — random-access roofline probes for MI355X (measurement tool,
// not product code).  Prices the access shapes the verdict kernels use:
//   k_gather64 : each lane reads one random 64-B line (4 x dwordx4) of a table
//   k_gather4  : each lane reads one random 4-B word
//   k_atomic8  : each lane does one 64-bit atomicAdd at a random 8-B slot
// Tables of a chosen size decide the tier (L2 4 MiB/XCD, Infinity Cache 256 MiB, HBM).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) k_gather64(const uint4 *t, uint64_t nlines, uint64_t n, uint32_t seed,
                                                  uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t l = mix(i ^ ((uint64_t)seed << 40)) % nlines;
        const uint4 *p = t + l * 4;
        uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc += a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// k_gather64 with the lines in ascending order: read i goes to line i * step + a random
// jitter below step (what sorting a batch's random lookups by address gives: the same
// lines, the same count, nearby addresses per wave)
__global__ void __launch_bounds__(256) k_gather64_sorted(const uint4 *t, uint64_t nlines, uint64_t n, uint32_t seed,
                                                         uint32_t *sink)
{
    const uint64_t step = nlines / n > 0 ? nlines / n : 1;
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t l = (i * step + mix(i ^ ((uint64_t)seed << 40)) % step) % nlines;
        const uint4 *p = t + l * 4;
        uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc += a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_gather4(const uint32_t *t, uint64_t nwords, uint64_t n, uint32_t seed,
                                                 uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        acc += t[mix(i ^ ((uint64_t)seed << 40)) % nwords];
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) k_atomic8(unsigned long long *t, uint64_t nslots, uint64_t n, uint32_t seed)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        atomicAdd(&t[mix(i ^ ((uint64_t)seed << 40)) % nslots], 1ull);
}

__global__ void __launch_bounds__(256) k_stream(const uint4 *t, uint64_t nvec, uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nvec; i += (uint64_t)gridDim.x * 256) {
        uint4 v = t[i];
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

extern "C" {
// kind: 0 gather64, 1 gather4, 2 atomic8, 3 stream, 4 gather64 sorted; returns kernel ms (median of reps)
float probe_run(int kind, uint64_t table_bytes, uint64_t n, int grid, int reps)
{
    void *t = nullptr, *sink = nullptr;
    if (hipMalloc(&t, table_bytes) != hipSuccess) return -1.f;
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(t, 1, table_bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipEventRecord(a, 0);
        if (kind == 0)
            hipLaunchKernelGGL(k_gather64, dim3(grid), dim3(256), 0, 0, (const uint4 *)t, table_bytes / 64, n, r,
                               (uint32_t *)sink);
        else if (kind == 1)
            hipLaunchKernelGGL(k_gather4, dim3(grid), dim3(256), 0, 0, (const uint32_t *)t, table_bytes / 4, n, r,
                               (uint32_t *)sink);
        else if (kind == 2)
            hipLaunchKernelGGL(k_atomic8, dim3(grid), dim3(256), 0, 0, (unsigned long long *)t, table_bytes / 8, n, r);
        else if (kind == 4)
            hipLaunchKernelGGL(k_gather64_sorted, dim3(grid), dim3(256), 0, 0, (const uint4 *)t, table_bytes / 64, n, r,
                               (uint32_t *)sink);
        else
            hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, (const uint4 *)t, table_bytes / 16,
                               (uint32_t *)sink);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms < best) best = ms;     // first run warms
    }
    (void)hipFree(t);
    (void)hipFree(sink);
    return best;
}
}

// ---- XCD-local atomics: one replica of the counter table per XCD, selected by
// HW_REG_XCC_ID; workgroup-scope atomics stay in the XCD's L2.
__device__ __forceinline__ uint32_t xcc_id()
{
    // s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0]
    return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xF;
}

__global__ void __launch_bounds__(256) k_atomic8_xcd(unsigned long long *t, uint64_t nslots, uint64_t n,
                                                     uint32_t seed, int scope)
{
    unsigned long long *rep = t + (uint64_t)xcc_id() * nslots;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        unsigned long long *p = &rep[mix(i ^ ((uint64_t)seed << 40)) % nslots];
        if (scope == 0) __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else __hip_atomic_fetch_add(p, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void k_xcc_map(uint32_t *out)
{
    if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

extern "C" {
// returns best ms; *sum_ok = 1 when Σ replicas == n * (reps + 1)
float probe_atomic_xcd(uint64_t nslots, uint64_t n, int grid, int reps, int scope, int *sum_ok)
{
    unsigned long long *t = nullptr;
    const uint64_t bytes = nslots * 8 * 16;
    if (hipMalloc(&t, bytes) != hipSuccess) return -1.f;
    (void)hipMemset(t, 0, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(k_atomic8_xcd, dim3(grid), dim3(256), 0, 0, t, nslots, n, r, scope);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r > 0 && ms < best) best = ms;
    }
    unsigned long long *h = (unsigned long long *)malloc(bytes);
    (void)hipMemcpy(h, t, bytes, hipMemcpyDeviceToHost);
    unsigned long long s = 0;
    for (uint64_t i = 0; i < nslots * 16; ++i) s += h[i];
    *sum_ok = s == n * (uint64_t)(reps + 1);
    free(h);
    (void)hipFree(t);
    return best;
}

int probe_xcc_map(int grid, uint32_t *out)
{
    uint32_t *d;
    (void)hipMalloc(&d, grid * 4);
    hipLaunchKernelGGL(k_xcc_map, dim3(grid), dim3(64), 0, 0, d);
    (void)hipMemcpy(out, d, grid * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return 0;
}
}
