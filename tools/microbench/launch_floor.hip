// Floor measurements for the march prologue on MI355X: an empty kernel, a store-only kernel with
// the march's lane->pixel mapping, and the same with a 3 KB LDS staging step, at the C3 grid
// (8100 workgroups of 256 threads).  Build: hipcc --offload-arch=gfx950 -O3 launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_empty(float4*) {}

__device__ __forceinline__ void pix(int& x, int& y) {
    const int tiles_y = (1080 + 15) / 16;
    const int tx = blockIdx.x / tiles_y, ty = blockIdx.x % tiles_y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    x = tx * 16 + (wave >> 1) * 8 + (lane >> 3);
    y = ty * 16 + (wave & 1) * 8 + (lane & 7);
}

__global__ __launch_bounds__(256) void k_store(float4* out) {
    int x, y;
    pix(x, y);
    if (x < 1920 && y < 1080) out[(size_t)x * 1080 + y] = make_float4(0.2f, 0.2f, 0.2f, 1.0f);
}

__global__ __launch_bounds__(256) void k_store_contig(float4* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < (size_t)1920 * 1080) out[i] = make_float4(0.2f, 0.2f, 0.2f, 1.0f);
}

__device__ __forceinline__ void st_nt(float4* p, float4 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
}

// the march's mapping with non-temporal stores (what the march kernels do)
__global__ __launch_bounds__(256) void k_store_nt(float4* out) {
    int x, y;
    pix(x, y);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4(0.2f, 0.2f, 0.2f, 1.0f));
}

// work tiles of 4 x 64 pixels: each wave stores one 64-pixel (1 KB) run of a frame column
__global__ __launch_bounds__(256) void k_store_col_nt(float4* out) {
    const int tiles_y = (1080 + 63) / 64;
    const int tx = blockIdx.x / tiles_y, ty = blockIdx.x % tiles_y;
    const int x = tx * 4 + (threadIdx.x >> 6), y = ty * 64 + (threadIdx.x & 63);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4(0.2f, 0.2f, 0.2f, 1.0f));
}

// 8 x 32 tiles, wave = 2 columns x 32 rows (512 B runs)
__global__ __launch_bounds__(256) void k_store_8x32_nt(float4* out) {
    const int tiles_y = (1080 + 31) / 32;
    const int tx = blockIdx.x / tiles_y, ty = blockIdx.x % tiles_y;
    const int x = tx * 8 + (threadIdx.x >> 5), y = ty * 32 + (threadIdx.x & 31);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4(0.2f, 0.2f, 0.2f, 1.0f));
}

__global__ __launch_bounds__(256) void k_contig_nt(float4* out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < (size_t)1920 * 1080) st_nt(out + i, make_float4(0.2f, 0.2f, 0.2f, 1.0f));
}

__global__ __launch_bounds__(256) void k_stage_store(float4* out, const int* maps) {
    __shared__ int s[768];
    for (int i = threadIdx.x; i < 768; i += 256) s[i] = maps[i];
    __syncthreads();
    int x, y;
    pix(x, y);
    if (x < 1920 && y < 1080) out[(size_t)x * 1080 + y] = make_float4((float)s[(x + y) % 768], 0.2f, 0.2f, 1.0f);
}

// the same staging + store with 512-thread workgroups of 16 x 32 pixels (half the workgroups)
__global__ __launch_bounds__(512) void k_stage_store512(float4* out, const int* maps) {
    __shared__ int s[768];
    for (int i = threadIdx.x; i < 768; i += 512) s[i] = maps[i];
    __syncthreads();
    const int tiles_y = (1080 + 31) / 32;
    const int tx = blockIdx.x / tiles_y, ty = blockIdx.x % tiles_y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = tx * 16 + (wave & 1) * 8 + (lane >> 3), y = ty * 32 + (wave >> 1) * 8 + (lane & 7);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4((float)s[(x + y) % 768], 0.2f, 0.2f, 1.0f));
}

__global__ __launch_bounds__(256) void k_stage_store_nt(float4* out, const int* maps) {
    __shared__ int s[768];
    for (int i = threadIdx.x; i < 768; i += 256) s[i] = maps[i];
    __syncthreads();
    int x, y;
    pix(x, y);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4((float)s[(x + y) % 768], 0.2f, 0.2f, 1.0f));
}

// The march prologue's dependent global round trips at the C3 grid: the work-tile load alone (dep1),
// then a per-ray table load that needs the tile (dep2: the fixed-axis map / column mask of
// init_ray), then a load that needs that one (dep3: the first class gather), each before the store
__device__ __forceinline__ void tile_pix(const int4 t, int& x, int& y) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    x = t.x + (wave & 1) * 8 + (lane >> 3);
    y = t.y + (wave >> 1) * 8 + (lane & 7);
}

__global__ __launch_bounds__(256) void k_dep1_nt(float4* out, const int4* tiles, const int* maps) {
    int x, y;
    tile_pix(tiles[blockIdx.x], x, y);
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4(0.2f, 0.2f, 0.2f, 1.0f));
}

__global__ __launch_bounds__(256) void k_dep2_nt(float4* out, const int4* tiles, const int* maps) {
    int x, y;
    tile_pix(tiles[blockIdx.x], x, y);
    const int m = maps[(x * 7 + y) & 767];
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4((float)m, 0.2f, 0.2f, 1.0f));
}

__global__ __launch_bounds__(256) void k_dep3_nt(float4* out, const int4* tiles, const int* maps) {
    int x, y;
    tile_pix(tiles[blockIdx.x], x, y);
    const int m = maps[(x * 7 + y) & 767];
    const int m2 = maps[(m + x) & 767];
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4((float)m2, 0.2f, 0.2f, 1.0f));
}

// dep2 with the staging of stage_store (3 KB into LDS + barrier) issued beside the tile load
__global__ __launch_bounds__(256) void k_dep2_stage_nt(float4* out, const int4* tiles, const int* maps) {
    __shared__ int s[768];
    const int4 t = tiles[blockIdx.x];
    int v[3];
    for (int u = 0; u < 3; ++u) v[u] = maps[threadIdx.x + 256 * u];
    int x, y;
    tile_pix(t, x, y);
    const int m = maps[(x * 7 + y) & 767];
    for (int u = 0; u < 3; ++u) s[threadIdx.x + 256 * u] = v[u];
    __syncthreads();
    if (x < 1920 && y < 1080) st_nt(out + (size_t)x * 1080 + y, make_float4((float)(m + s[(x + y) % 768]), 0.2f, 0.2f, 1.0f));
}

int main() {
    float4* out;
    int* maps;
    CK(hipMalloc(&out, (size_t)1920 * 1080 * 16));
    CK(hipMalloc(&maps, 768 * 4));
    CK(hipMemset(maps, 0, 768 * 4));
    const int nwg = (1920 / 16) * ((1080 + 15) / 16);
    int4* tiles;
    {
        std::vector<int4> h(nwg);
        const int ty_n = (1080 + 15) / 16;
        for (int i = 0; i < nwg; ++i) h[i] = make_int4((i / ty_n) * 16, (i % ty_n) * 16, 0, 0);
        CK(hipMalloc(&tiles, nwg * sizeof(int4)));
        CK(hipMemcpy(tiles, h.data(), nwg * sizeof(int4), hipMemcpyHostToDevice));
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        const int n = 200;
        for (int i = 0; i < n; ++i) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("%-28s %8.2f us / launch\n", name, ms * 1000.0f / n);
        return 0;
    };
    run("empty 8100x256", [&] { hipLaunchKernelGGL(k_empty, dim3(nwg), dim3(256), 0, 0, out); });
    run("store march mapping", [&] { hipLaunchKernelGGL(k_store, dim3(nwg), dim3(256), 0, 0, out); });
    run("store contiguous", [&] { hipLaunchKernelGGL(k_store_contig, dim3(nwg), dim3(256), 0, 0, out); });
    run("store march mapping nt", [&] { hipLaunchKernelGGL(k_store_nt, dim3(nwg), dim3(256), 0, 0, out); });
    run("store 4x64 tiles nt", [&] { hipLaunchKernelGGL(k_store_col_nt, dim3(480 * 17), dim3(256), 0, 0, out); });
    run("store 8x32 tiles nt", [&] { hipLaunchKernelGGL(k_store_8x32_nt, dim3(240 * 34), dim3(256), 0, 0, out); });
    run("store contiguous nt", [&] { hipLaunchKernelGGL(k_contig_nt, dim3(nwg), dim3(256), 0, 0, out); });
    run("stage 3KB + store", [&] { hipLaunchKernelGGL(k_stage_store, dim3(nwg), dim3(256), 0, 0, out, maps); });
    run("stage 3KB + store nt", [&] { hipLaunchKernelGGL(k_stage_store_nt, dim3(nwg), dim3(256), 0, 0, out, maps); });
    run("stage 3KB + store nt 512", [&] { hipLaunchKernelGGL(k_stage_store512, dim3(120 * 34), dim3(512), 0, 0, out, maps); });
    run("dep1: tile load + store nt", [&] { hipLaunchKernelGGL(k_dep1_nt, dim3(nwg), dim3(256), 0, 0, out, tiles, maps); });
    run("dep2: + ray load", [&] { hipLaunchKernelGGL(k_dep2_nt, dim3(nwg), dim3(256), 0, 0, out, tiles, maps); });
    run("dep3: + dependent load", [&] { hipLaunchKernelGGL(k_dep3_nt, dim3(nwg), dim3(256), 0, 0, out, tiles, maps); });
    run("dep2 + 3KB staging", [&] { hipLaunchKernelGGL(k_dep2_stage_nt, dim3(nwg), dim3(256), 0, 0, out, tiles, maps); });
    run("empty 2025x1024", [&] { hipLaunchKernelGGL(k_empty, dim3(nwg / 4), dim3(1024), 0, 0, out); });
    return 0;
}
