// membench8.hip -- HBM ceilings on MI355X for round 4's two questions (tools/gpu_membench8.sh):
//
//  1. the copy ceiling bench.py reports (gs_stream_copy): grid-stride 16-B copies with U loads in flight per
//     lane, plain or non-temporal (__builtin_nontemporal_load/store), and wave-contiguous chunks;
//  2. the 8-bit pass-1 shape (GS_HB8 + GS_MV8): one workgroup per exchange (a, b) of random distinct rows of
//     two [R][NC] u8 matrices (heartbeat and max_version views), reading both rows of both matrices plus an
//     L2-resident per-owner u16 word per column, writing both heartbeat rows back, at C columns per lane per
//     group, A groups in flight ahead, W waves per exchange, compiled for O waves per SIMD.
//
// Prints one line per variant: ms per launch and GB/s of (read + write) HBM bytes over HIP-event time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // native vector: the nontemporal builtins take it
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_gs(v4u *__restrict__ dst, const v4u *__restrict__ src, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// each wave copies contiguous 16 KiB chunks (64 lanes x 16 B x 16), chunks dealt grid-stride over the waves
template <bool NT>
__global__ __launch_bounds__(256) void copy_chunk(v4u *__restrict__ dst, const v4u *__restrict__ src, uint64_t n) {
    const uint64_t waves = (uint64_t)gridDim.x * 4u, wid = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t chunks = n / 1024u;
    for (uint64_t c = wid; c < chunks; c += waves) {
        const uint64_t b = c * 1024u + lane;
        v4u v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = NT ? __builtin_nontemporal_load(src + b + u * 64) : src[b + u * 64];
#pragma unroll
        for (int u = 0; u < 16; u++) {
            if (NT) __builtin_nontemporal_store(v[u], dst + b + u * 64);
            else dst[b + u * 64] = v[u];
        }
    }
}

template <int C>
struct Vec;
template <>
struct Vec<4> { using T = uint32_t; using P = uint2; };
template <>
struct Vec<8> { using T = v2u; using P = uint4; };
template <>
struct Vec<16> { using T = v4u; using P = uint4; };  // P: 2 x uint4 for 16 columns (loaded as two)

__device__ __forceinline__ uint32_t bmax(uint32_t x, uint32_t y) {  // byte-wise stand-in merge (SWAR select)
    const uint32_t d = ((x | 0x80808080u) - (y & 0x7F7F7F7Fu)) & 0x80808080u;
    const uint32_t m = (d >> 7) * 0xFFu;
    return (x & m) | (y & ~m);
}

// one group: C columns per lane of the four rows + the per-owner words
template <int C>
struct G8 {
    uint32_t a[C / 4], b[C / 4], ma[C / 4], mb[C / 4], p[C / 2];
};
template <int C, bool NT>
__device__ __forceinline__ void ld_g8(const uint8_t *hA, const uint8_t *hB, const uint8_t *mA, const uint8_t *mB,
                                      const uint16_t *own, uint32_t c, G8<C> &g) {
    using T = typename Vec<C>::T;
    auto ld = [&](const uint8_t *p, uint32_t *o) {
        const T v = NT ? __builtin_nontemporal_load(reinterpret_cast<const T *>(p + c)) : *reinterpret_cast<const T *>(p + c);
        __builtin_memcpy(o, &v, sizeof v);
    };
    ld(hA, g.a);
    ld(hB, g.b);
    ld(mA, g.ma);
    ld(mB, g.mb);
    if (C == 4) {
        const uint2 v = *reinterpret_cast<const uint2 *>(own + c);
        g.p[0] = v.x; g.p[1] = v.y;
    } else {
#pragma unroll
        for (int q = 0; q < C / 8; q++) {
            const uint4 v = *reinterpret_cast<const uint4 *>(own + c + 8 * q);
            g.p[4 * q] = v.x; g.p[4 * q + 1] = v.y; g.p[4 * q + 2] = v.z; g.p[4 * q + 3] = v.w;
        }
    }
}

template <int C, int A, int W, int O, bool NT>
__global__ __launch_bounds__(64 * W, O) void pass8(uint8_t *hb, const uint8_t *mv, const uint16_t *own, const int *pa,
                                                   const int *pb, uint32_t NC, unsigned *sink) {
    using T = typename Vec<C>::T;
    const size_t ra = (size_t)pa[blockIdx.x] * NC, rb = (size_t)pb[blockIdx.x] * NC;
    const uint8_t *hA = hb + ra, *hB = hb + rb, *mA = mv + ra, *mB = mv + rb;
    const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t span = NC / W, lo = wid * span, hi = lo + span;  // this wave's part of the row
    constexpr uint32_t STEP = 64u * C;
    uint32_t acc = 0;
    G8<C> g[A + 1];
    uint32_t c = lo + lane * C;
#pragma unroll
    for (int k = 0; k < A; k++)
        if (c + k * STEP < hi) ld_g8<C, NT>(hA, hB, mA, mB, own, c + k * STEP, g[k]);
    while (c < hi) {
        if (c + A * STEP < hi) ld_g8<C, NT>(hA, hB, mA, mB, own, c + A * STEP, g[A]);
        G8<C> &x = g[0];
        uint32_t na[C / 4];
#pragma unroll
        for (int q = 0; q < C / 4; q++) {
            na[q] = bmax(x.a[q], x.b[q]);
            acc += __popc(((x.ma[q] | 0x80808080u) - (x.mb[q] & 0x7F7F7F7Fu)) & 0x80808080u) + (x.p[q / 2] & 1u);
        }
        T w;
        __builtin_memcpy(&w, na, sizeof w);
        *reinterpret_cast<T *>(hb + ra + c) = w;
        *reinterpret_cast<T *>(hb + rb + c) = w;
#pragma unroll
        for (int k = 0; k < A; k++) g[k] = g[k + 1];
        c += STEP;
    }
    if (acc == 0x9E3779B9u) atomicAdd(sink, 1u);
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main() {
    {
        const uint64_t bytes = 4ull << 30, n16 = bytes / 16;
        v4u *src, *dst;
        CK(hipMalloc(&src, bytes));
        CK(hipMalloc(&dst, bytes));
        CK(hipMemset(src, 1, bytes));
        CK(hipMemset(dst, 0, bytes));
        const int reps = 8;
        auto rep = [&](const char *name, float ms) { printf("%-34s %.3f ms %6.0f GB/s\n", name, ms, 2.0 * bytes / (ms * 1e6)); };
        rep("copy_gs U=8 G=32768", timeit([&] { copy_gs<8, false><<<32768, 256>>>(dst, src, n16); }, reps));
        rep("copy_gs U=8 G=32768 nt", timeit([&] { copy_gs<8, true><<<32768, 256>>>(dst, src, n16); }, reps));
        rep("copy_gs U=4 G=65536 nt", timeit([&] { copy_gs<4, true><<<65536, 256>>>(dst, src, n16); }, reps));
        rep("copy_gs U=16 G=8192 nt", timeit([&] { copy_gs<16, true><<<8192, 256>>>(dst, src, n16); }, reps));
        rep("copy_gs U=8 G=4096 nt", timeit([&] { copy_gs<8, true><<<4096, 256>>>(dst, src, n16); }, reps));
        rep("copy_chunk G=2048", timeit([&] { copy_chunk<false><<<2048, 256>>>(dst, src, n16); }, reps));
        rep("copy_chunk G=2048 nt", timeit([&] { copy_chunk<true><<<2048, 256>>>(dst, src, n16); }, reps));
        rep("copy_chunk G=8192 nt", timeit([&] { copy_chunk<true><<<8192, 256>>>(dst, src, n16); }, reps));
        rep("copy_chunk G=65536 nt", timeit([&] { copy_chunk<true><<<65536, 256>>>(dst, src, n16); }, reps));
        rep("hipMemcpyDtoD", timeit([&] { CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0)); }, reps));
        CK(hipFree(dst));
        CK(hipFree(src));
    }
    // the headline's pass-1 shape: 65,536 rows x 65,536 u8 columns x 2 matrices (8 GiB), 19,800 disjoint
    // random pairs (one phase), per-owner u16 words (128 KiB, L2-resident)
    const uint32_t R = 65536, NC = 65536, P = 19800;
    uint8_t *hb, *mv;
    uint16_t *own;
    int *pa, *pb;
    unsigned *sink;
    CK(hipMalloc(&hb, (size_t)R * NC));
    CK(hipMalloc(&mv, (size_t)R * NC));
    CK(hipMalloc(&own, NC * 2));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(hb, 3, (size_t)R * NC));
    CK(hipMemset(mv, 5, (size_t)R * NC));
    CK(hipMemset(own, 7, NC * 2));
    std::vector<int> perm(R);
    for (uint32_t i = 0; i < R; i++) perm[i] = (int)i;
    srand(7);
    for (uint32_t i = R - 1; i > 0; i--) std::swap(perm[i], perm[rand() % (i + 1)]);
    std::vector<int> ha(perm.begin(), perm.begin() + P), hbv(perm.begin() + P, perm.begin() + 2 * P);
    CK(hipMalloc(&pa, P * 4));
    CK(hipMalloc(&pb, P * 4));
    CK(hipMemcpy(pa, ha.data(), P * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(pb, hbv.data(), P * 4, hipMemcpyHostToDevice));
    const double moved = (double)P * NC * (4 + 2);  // read 2 matrices x 2 rows, write 1 matrix x 2 rows
    const int reps = 10;
#define PASS8(C, A, W, O, NT)                                                                                   \
    do {                                                                                                        \
        const float ms = timeit([&] { pass8<C, A, W, O, NT><<<P, 64 * W>>>(hb, mv, own, pa, pb, NC, sink); }, reps); \
        printf("pass8 C=%2d A=%d W=%d O=%d nt=%d   %.3f ms %6.0f GB/s\n", C, A, W, O, (int)NT, ms, moved / (ms * 1e6)); \
    } while (0)
    PASS8(4, 2, 2, 5, false);  // round 3's shape: 4 columns per lane, 2 groups ahead, 5 waves per SIMD
    PASS8(4, 2, 2, 8, false);
    PASS8(8, 1, 2, 8, false);
    PASS8(8, 2, 2, 6, false);
    PASS8(16, 1, 2, 8, false);
    PASS8(16, 1, 2, 6, false);
    PASS8(16, 2, 2, 4, false);
    PASS8(16, 1, 4, 8, false);
    PASS8(16, 1, 2, 8, true);
    PASS8(16, 0, 2, 8, false);
    PASS8(8, 0, 2, 8, false);
    PASS8(16, 1, 8, 8, false);
    return 0;
}
