// FETCH_SIZE calibration for K2's access patterns (MI355X_MICROARCH.md: "calibrate on
// a known byte count in your own access pattern before trusting an absolute").
// Reads a known number of bytes with (a) non-temporal 16-B/lane loads, (b) plain
// 16-B/lane loads, (c) K2's row pattern (lane k reads 64-B record k with four 16-B
// loads), and (d) K2's flattened-stream pattern (consecutive 16-B chunks of many
// segments whose starts are 16-B but not line aligned).  Run under
// rocprofv3 --pmc FETCH_SIZE; compare FETCH_SIZE x 2 x 1 KiB with the bytes printed.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256ull) {
        u32x4 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x * 256 + threadIdx.x] = acc;  // never true on a zeroed buffer
}

// lane k of each wave reads record (item * 64 + k): four 16-B loads at stride 64 B
__global__ __launch_bounds__(256) void k_rows(const u32x4* __restrict__ rows, uint64_t nrec, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t r = blockIdx.x * 256ull + threadIdx.x; r < nrec; r += (uint64_t)gridDim.x * 256ull) {
        const u32x4* q = rows + 4 * r;
        u32x4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc ^= a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// segments of `seg` 16-B chunks placed back to back with a `gap`-chunk hole after
// each (the hole is never read): each wave streams 64 x 4 consecutive chunks of the
// read space per pass with NT loads, like k_compare_flat over [A][B] blobs
__global__ __launch_bounds__(256) void k_segs(const u32x4* __restrict__ p, uint64_t nseg, uint32_t seg, uint32_t gap,
                                              uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t total = nseg * seg;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * 4;
    for (uint64_t base = wave * 256; base < total; base += nw * 256) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t g = base + u * 64 + lane;
            if (g < total) {
                const uint64_t s = g / seg, k = g % seg;
                u32x4 v = __builtin_nontemporal_load(p + s * (seg + gap) + k);
                acc ^= v.x ^ v.w;
            }
        }
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// K2's two interleaved streams: pair i = [A_i][B_i], each blob `seg` chunks at a
// stride of `stride` chunks (stride - seg = padding, never read); flattened over
// the pairs' chunks, each lane loads chunk k of A and of B (NT), like k_compare_flat
__global__ __launch_bounds__(256) void k_pairs(const u32x4* __restrict__ p, uint64_t npairs, uint32_t seg,
                                               uint32_t stride, uint32_t* out) {
    uint32_t acc = 0;
    const uint64_t total = npairs * seg;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6, nw = (uint64_t)gridDim.x * 4;
    for (uint64_t base = wave * 256; base < total; base += nw * 256) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t g = base + u * 64 + lane;
            if (g < total) {
                const uint64_t s = g / seg, k = g % seg;
                const u32x4* a = p + s * 2 * stride + k;
                u32x4 va = __builtin_nontemporal_load(a), vb = __builtin_nontemporal_load(a + stride);
                acc ^= va.x ^ vb.w;
            }
        }
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const uint64_t bytes = 8ull << 30;
    u32x4* buf;
    uint32_t* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
    if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const int grid = 4096;
    for (int r = 0; r < 3; r++) {
        k_read<true><<<grid, 256>>>(buf, bytes / 16, out);
        k_read<false><<<grid, 256>>>(buf, bytes / 16, out);
        k_rows<<<grid, 256>>>(buf, (640ull << 20) / 64, out);
        // 201-chunk segments (a ~3.2 KB blob) with a 1-chunk hole: 16-B aligned starts
        k_segs<<<grid, 256>>>(buf, (bytes / 16) / 202, 201, 1, out);
        // the same loop over one contiguous range (no holes), and over 128-B aligned 3200-B segments
        k_segs<<<grid, 256>>>(buf, (bytes / 16) / 202, 202, 0, out);
        k_segs<<<grid, 256>>>(buf, (bytes / 16) / 208, 200, 8, out);
        // start line-aligned, end partial
        k_segs<<<grid, 256>>>(buf, (bytes / 16) / 208, 201, 7, out);
        // K2's pattern: 16-B packed blobs; 128-B aligned starts with partial ends; fully aligned
        k_pairs<<<grid, 256>>>(buf, (bytes / 16) / 402, 201, 201, out);
        k_pairs<<<grid, 256>>>(buf, (bytes / 16) / 416, 201, 208, out);
        k_pairs<<<grid, 256>>>(buf, (bytes / 16) / 416, 200, 208, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("k_read: %llu bytes per launch\n", (unsigned long long)bytes);
    printf("k_rows: %llu bytes per launch\n", (unsigned long long)(640ull << 20));
    printf("k_segs 201+1: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 202) * 201 * 16));
    printf("k_segs 202+0: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 202) * 202 * 16));
    printf("k_segs 200+8: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 208) * 200 * 16));
    printf("k_segs 201+7: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 208) * 201 * 16));
    printf("k_pairs 201/201: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 402) * 402 * 16));
    printf("k_pairs 201/208: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 416) * 402 * 16));
    printf("k_pairs 200/208: %llu bytes per launch\n", (unsigned long long)(((bytes / 16) / 416) * 400 * 16));
    return 0;
}
