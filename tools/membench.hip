// membench.hip -- HBM ceilings on MI355X for the shapes this repo's kernels stream (tools/membench.sh).
//
//  copy_gs<U>   grid-stride 16-B-per-lane copy, U loads in flight per lane, G blocks
//  copy_tile    one 256-thread block copies one 64 KiB tile (16 loads of 16 B per lane in flight)
//  read_tile    the same tile shape, read only
//  rowpair<V>   k_pass1's shape: one 128-thread workgroup per (a, b) pair of random rows of an
//               [R][NC] u16 matrix pair (heartbeats, max versions); reads both arrays of both rows and
//               writes the heartbeat array of both rows back; V = bytes per lane per array (8 or 16)
//
// Prints one line per variant: GB/s of (read + write) bytes over HIP-event time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void copy_gs(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) dst[i + u * stride] = v[u];
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void copy_tile(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096u + threadIdx.x;  // 64 KiB per block
    uint4 v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) v[u] = base + u * 256u < n ? src[base + u * 256u] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 16; u++)
        if (base + u * 256u < n) dst[base + u * 256u] = v[u];
}

__global__ __launch_bounds__(256) void read_tile(const uint4 *__restrict__ src, uint64_t n, unsigned *sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096u + threadIdx.x;
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < 16; u++)
        if (base + u * 256u < n) {
            const uint4 v = src[base + u * 256u];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    if (acc == 0x9E3779B9u) atomicAdd(sink, 1u);
}

// V = 8: uint2 (4 columns) per lane per array; V = 16: uint4 (8 columns).  Next step's loads issued
// before this step's stores (k_pass1's software pipeline).
template <int V>
__global__ __launch_bounds__(128) void rowpair(uint16_t *hb, const uint16_t *mv, const int *pa, const int *pb,
                                               uint32_t NC) {
    using T = typename std::conditional<V == 8, uint2, uint4>::type;
    constexpr int CPL = V / 2;  // columns per lane
    const size_t ra = (size_t)pa[blockIdx.x] * NC, rb = (size_t)pb[blockIdx.x] * NC;
    const T *hA = reinterpret_cast<const T *>(hb + ra), *hB = reinterpret_cast<const T *>(hb + rb);
    const T *mA = reinterpret_cast<const T *>(mv + ra), *mB = reinterpret_cast<const T *>(mv + rb);
    T *wA = reinterpret_cast<T *>(hb + ra), *wB = reinterpret_cast<T *>(hb + rb);
    const uint32_t nv = NC / CPL;
    uint32_t i = threadIdx.x;
    T a0, b0, c0, d0;
    if (i < nv) { a0 = hA[i]; b0 = hB[i]; c0 = mA[i]; d0 = mB[i]; }
    while (i < nv) {
        const uint32_t i1 = i + 128u;
        T a1, b1, c1, d1;
        if (i1 < nv) { a1 = hA[i1]; b1 = hB[i1]; c1 = mA[i1]; d1 = mB[i1]; }
        // stand-in merge: max of the heartbeats, max versions folded in so the loads stay live
        T x, y;
        const uint32_t *pa0 = reinterpret_cast<const uint32_t *>(&a0), *pb0 = reinterpret_cast<const uint32_t *>(&b0);
        const uint32_t *pc0 = reinterpret_cast<const uint32_t *>(&c0), *pd0 = reinterpret_cast<const uint32_t *>(&d0);
        uint32_t *px = reinterpret_cast<uint32_t *>(&x), *py = reinterpret_cast<uint32_t *>(&y);
#pragma unroll
        for (int q = 0; q < V / 4; q++) {
            px[q] = max(pa0[q], pb0[q]) ^ (pc0[q] & 0x8000u);
            py[q] = max(pa0[q], pb0[q]) ^ (pd0[q] & 0x8000u);
        }
        wA[i] = x;
        wB[i] = y;
        a0 = a1; b0 = b1; c0 = c1; d0 = d1;
        i = i1;
    }
}

// scatter: one 2-byte store per lane to arbitrary positions of a large u16 array (the packer's
// max_version applies: ~570 sparse columns of one receiver row per exchange direction)
__global__ __launch_bounds__(256) void scatter16(uint16_t *a, const uint64_t *pos, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n) a[pos[i]] = (uint16_t)i;
}
__global__ __launch_bounds__(256) void gather16(const uint16_t *a, const uint64_t *pos, uint64_t n, unsigned *sink) {
    const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (i < n && a[pos[i]] == 0x1234u) atomicAdd(sink, 1u);
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
    const uint64_t bytes = 4ull << 30;
    const uint64_t n16 = bytes / 16;
    uint4 *src, *dst;
    unsigned *sink;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(src, 1, bytes));
    CK(hipMemset(dst, 0, bytes));
    const int reps = 10;
    for (int G : {2048, 8192, 32768}) {
        float ms = timeit([&] { copy_gs<4><<<G, 256>>>(dst, src, n16); }, reps);
        printf("copy_gs U=4 G=%d: %.0f GB/s\n", G, 2.0 * bytes / (ms * 1e6));
        ms = timeit([&] { copy_gs<8><<<G, 256>>>(dst, src, n16); }, reps);
        printf("copy_gs U=8 G=%d: %.0f GB/s\n", G, 2.0 * bytes / (ms * 1e6));
    }
    const uint32_t tiles = (uint32_t)((n16 + 4095) / 4096);
    float ms = timeit([&] { copy_tile<<<tiles, 256>>>(dst, src, n16); }, reps);
    printf("copy_tile 64KiB/block: %.0f GB/s\n", 2.0 * bytes / (ms * 1e6));
    ms = timeit([&] { read_tile<<<tiles, 256>>>(src, n16, sink); }, reps);
    printf("read_tile 64KiB/block: %.0f GB/s (read only)\n", 1.0 * bytes / (ms * 1e6));
    CK(hipFree(dst));
    CK(hipFree(src));

    // k_pass1 shape: 65,536 rows x 65,536 u16 columns x 2 arrays (16 GiB), 19,800 disjoint random pairs
    const uint32_t R = 65536, NC = 65536, P = 19800;
    uint16_t *hb, *mv;
    int *pa, *pb;
    CK(hipMalloc(&hb, (size_t)R * NC * 2));
    CK(hipMalloc(&mv, (size_t)R * NC * 2));
    CK(hipMemset(hb, 3, (size_t)R * NC * 2));
    CK(hipMemset(mv, 5, (size_t)R * NC * 2));
    std::vector<int> perm(R);
    for (uint32_t i = 0; i < R; i++) perm[i] = (int)i;
    srand(7);
    for (uint32_t i = R - 1; i > 0; i--) std::swap(perm[i], perm[rand() % (i + 1)]);
    std::vector<int> ha(perm.begin(), perm.begin() + P), hbv(perm.begin() + P, perm.begin() + 2 * P);
    CK(hipMalloc(&pa, P * 4));
    CK(hipMalloc(&pb, P * 4));
    CK(hipMemcpy(pa, ha.data(), P * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(pb, hbv.data(), P * 4, hipMemcpyHostToDevice));
    const double moved = (double)P * NC * 2 * (4 + 2);  // read 2 arrays x 2 rows, write 1 array x 2 rows
    ms = timeit([&] { rowpair<8><<<P, 128>>>(hb, mv, pa, pb, NC); }, reps);
    printf("rowpair 8 B/lane: %.3f ms, %.0f GB/s\n", ms, moved / (ms * 1e6));
    ms = timeit([&] { rowpair<16><<<P, 128>>>(hb, mv, pa, pb, NC); }, reps);
    printf("rowpair 16 B/lane: %.3f ms, %.0f GB/s\n", ms, moved / (ms * 1e6));

    // packer applies: 19,800 exchanges x 2 directions x ~570 sparse columns of the receiver row, sorted
    // within a row (as the packer issues them), into the [R][NC] u16 max_version matrix
    {
        const uint32_t per = 570;
        const uint64_t S = (uint64_t)P * 2 * per;
        std::vector<uint64_t> pos(S);
        uint64_t k = 0;
        for (uint32_t e = 0; e < P; e++)
            for (int dir = 0; dir < 2; dir++) {
                const uint64_t row = dir ? hbv[e] : ha[e];
                std::vector<uint32_t> cols(per);
                for (auto &c : cols) c = (uint32_t)(rand() % NC);
                std::sort(cols.begin(), cols.end());
                for (auto c : cols) pos[k++] = row * NC + c;
            }
        uint64_t *dpos;
        CK(hipMalloc(&dpos, S * 8));
        CK(hipMemcpy(dpos, pos.data(), S * 8, hipMemcpyHostToDevice));
        const uint32_t blocks = (uint32_t)((S + 255) / 256);
        ms = timeit([&] { scatter16<<<blocks, 256>>>(mv, dpos, S); }, reps);
        printf("scatter 2-B stores (%llu, row-sorted): %.3f ms, %.1f G stores/s\n", (unsigned long long)S, ms,
               S / (ms * 1e6));
        ms = timeit([&] { gather16<<<blocks, 256>>>(mv, dpos, S, sink); }, reps);
        printf("gather 2-B loads (%llu, row-sorted): %.3f ms, %.1f G loads/s\n", (unsigned long long)S, ms,
               S / (ms * 1e6));
        // fully random order (no locality between neighbouring lanes)
        for (uint64_t i = S - 1; i > 0; i--) std::swap(pos[i], pos[rand() % (i + 1)]);
        CK(hipMemcpy(dpos, pos.data(), S * 8, hipMemcpyHostToDevice));
        ms = timeit([&] { scatter16<<<blocks, 256>>>(mv, dpos, S); }, reps);
        printf("scatter 2-B stores (random order): %.3f ms, %.1f G stores/s\n", ms, S / (ms * 1e6));
    }
    return 0;
}
