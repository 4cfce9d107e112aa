// gather_ceiling.hip - the measured ceiling of the traversal's memory pattern on this GPU.
//
// The trace kernels fetch 48-64-byte records (BVH nodes, triangles) at data-dependent
// addresses, every lane of a wave at a different one, from a scene that stays in L2 / the
// Infinity Cache.  This probe runs that pattern alone: a persistent grid like the walk's
// (256-thread workgroups, the walk's occupancy), every lane chasing a chain of random records
// of R bytes (R / 16 buffer_load_dwordx4 per record, as innerStep issues them) in a table of
// S bytes.  It prints the sustained record-bytes per second, the ceiling the walk's
// algorithmic bytes are compared with (bench.py roofline).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/build/gather_ceiling tools/gather_ceiling.hip
// run:   tools/build/gather_ceiling  (JSON lines on stdout)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// kChain: the next record index depends on the loaded data (the walk's dependent fetches);
// kCoherent: every lane of a wave fetches the same record (a perfectly coherent packet)
template <int kVec4, bool kCoherent>
__global__ __launch_bounds__(256, 1) void k_gather(const uint4* __restrict__ table, uint32_t nRecords, int iters,
                                                   uint32_t* out) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(table), static_cast<short>(0), 0x7FFFFFFF,
                                                       0x00020000);
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t idx = mix(kCoherent ? (tid >> 6) : tid) % nRecords;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < kVec4; ++k) {
            const uint4 v = __builtin_bit_cast(
                uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, (idx * kVec4 + k) * 16u, 0, 0));
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        acc += x;
        idx = mix(idx ^ x ^ static_cast<uint32_t>(i)) % nRecords;  // dependent next fetch
    }
    out[tid] = acc;
}

// The walk's node fetch on 64-B aligned records: three 16-B loads (the child boxes) and, with
// kRefs, the 8-B child-reference load at +48 - what a node whose references are folded into the
// boxes would save.
template <bool kRefs>
__global__ __launch_bounds__(256, 1) void k_gather_node(const uint4* __restrict__ table, uint32_t nRecords, int iters,
                                                       uint32_t* out) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(table), static_cast<short>(0), 0x7FFFFFFF,
                                                       0x00020000);
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t idx = mix(tid) % nRecords;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, idx * 64u + k * 16u, 0, 0));
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        if (kRefs) {
            const auto r = __builtin_amdgcn_raw_buffer_load_b64(rsrc, idx * 64u + 48u, 0, 0);
            x ^= static_cast<uint32_t>(r[0]) ^ static_cast<uint32_t>(r[1]);
        }
        acc += x;
        idx = mix(idx ^ x ^ static_cast<uint32_t>(i)) % nRecords;
    }
    out[tid] = acc;
}

// Quad-cooperative form of the divergent chase (64-B records): in round k the four lanes of a
// quad fetch the four 16-B pieces of lane (4q + k)'s record with one LDS-DMA load
// (global_load_lds_dwordx4), so one wave instruction touches 16 lines, 4 lanes each, instead of
// 64 lines; the record of lane 4q + k lands contiguously at round k's base + 64 q, and each
// lane reads its own record back with ds_read_b128.  Rounds are padded by 16 B (bank spread).
__global__ __launch_bounds__(256, 1) void k_gather_quad(const uint4* __restrict__ table, uint32_t nRecords, int iters,
                                                       uint32_t* out) {
    constexpr int kRound = 65;  // uint4 per round: 64 lanes + 1 pad
    __shared__ uint4 stage[4][4 * kRound];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = static_cast<int>(threadIdx.x & 63u), wave = static_cast<int>(threadIdx.x >> 6);
    uint32_t idx = mix(tid) % nRecords;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t ik[4];
        ik[0] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(idx), 0x00, 0xF, 0xF, false));
        ik[1] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(idx), 0x55, 0xF, 0xF, false));
        ik[2] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(idx), 0xAA, 0xF, 0xF, false));
        ik[3] = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(idx), 0xFF, 0xF, 0xF, false));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4* g = table + ik[k] * 4u + static_cast<uint32_t>(lane & 3);
            __builtin_amdgcn_global_load_lds(g, &stage[wave][k * kRound], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint4* mine = &stage[wave][(lane & 3) * kRound + (lane >> 2) * 4];
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = mine[k];
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        acc += x;
        idx = mix(idx ^ x ^ static_cast<uint32_t>(i)) % nRecords;
    }
    out[tid] = acc;
}

template <int kVec4, bool kCoherent, bool kQuad = false, int kNode = 0>
void run(size_t tableBytes, int blocksPerCU, const char* label) {
    int dev = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, dev));
    const uint32_t recBytes = 16u * kVec4;
    const uint32_t nRecords = static_cast<uint32_t>(tableBytes / recBytes);
    std::vector<uint32_t> host(tableBytes / 4);
    for (size_t i = 0; i < host.size(); ++i) host[i] = static_cast<uint32_t>(i * 2654435761u);
    uint4* table;
    uint32_t* out;
    const int blocks = prop.multiProcessorCount * blocksPerCU;
    CK(hipMalloc(&table, tableBytes));
    CK(hipMalloc(&out, sizeof(uint32_t) * blocks * 256));
    CK(hipMemcpy(table, host.data(), tableBytes, hipMemcpyHostToDevice));
    const int iters = 2000;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto launch = [&](int it) {
        if (kNode == 1)
            hipLaunchKernelGGL(k_gather_node<false>, dim3(blocks), dim3(256), 0, 0, table, nRecords, it, out);
        else if (kNode == 2)
            hipLaunchKernelGGL(k_gather_node<true>, dim3(blocks), dim3(256), 0, 0, table, nRecords, it, out);
        else if (kQuad)
            hipLaunchKernelGGL(k_gather_quad, dim3(blocks), dim3(256), 0, 0, table, nRecords, it, out);
        else
            hipLaunchKernelGGL((k_gather<kVec4, kCoherent>), dim3(blocks), dim3(256), 0, 0, table, nRecords, it, out);
    };
    launch(50);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(a, 0));
        launch(iters);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
    }
    const double lanes = static_cast<double>(blocks) * 256.0;
    const double bytes = lanes * iters * recBytes;
    std::printf("{\"pattern\": \"%s\", \"record_bytes\": %u, \"table_mib\": %.1f, \"blocks_per_cu\": %d, "
                "\"ms\": %.4f, \"gb_per_s\": %.1f, \"grecords_per_s\": %.3f}\n",
                label, recBytes, tableBytes / 1048576.0, blocksPerCU, best, bytes / (best * 1e-3) / 1e9,
                lanes * iters / (best * 1e-3) / 1e9);
    std::fflush(stdout);
    CK(hipFree(table));
    CK(hipFree(out));
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "node") {  // 64-B node records: 48 B vs 56 B fetched
        for (size_t mib : {8, 16, 32}) {
            run<4, false, false, 2>(mib << 20, 6, "node-48+8");
            run<4, false, false, 1>(mib << 20, 6, "node-48");
        }
        return 0;
    }
    // the walk: 6 workgroups of 256 threads per CU; Conference scene ~30 MB (nodes + triangles)
    for (size_t mib : {4, 32, 128}) {
        run<4, false>(mib << 20, 6, "divergent");
        run<3, false>(mib << 20, 6, "divergent");
        run<1, false>(mib << 20, 6, "divergent");
    }
    run<4, true>(32u << 20, 6, "wave-coherent");
    for (size_t mib : {4, 32, 128}) run<4, false, true>(mib << 20, 6, "quad-cooperative-lds-dma");
    run<4, false, true>(32u << 20, 4, "quad-cooperative-lds-dma");
    run<4, false>(32u << 20, 8, "divergent");
    return 0;
}
