// Probe: does an LDS-DMA (buffer_load_dwordx4 ... lds) land at LDS byte offsets above 128 KiB?
// One workgroup of 64 threads with a 152 KiB static LDS array: LDS is first filled with a marker
// by ordinary ds_write, then one wave DMAs a 1 KiB piece of a known pattern to each probe offset,
// and every 16-byte slot of LDS is copied out.  The host reports, per probe offset, whether the
// pattern landed there and whether it landed somewhere else (e.g. the offset modulo 128 KiB).
// Build: hipcc --offload-arch=gfx950 -O2 -o lds_dma_probe scripts/lds_dma_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int LDS_BYTES = 152 * 1024;
typedef __attribute__((address_space(3))) void lds_t;

__global__ __launch_bounds__(64) void probe(const uint32_t* src, int dst_off, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_BYTES / 4];
  const int lane = threadIdx.x;
  for (int i = lane; i < LDS_BYTES / 4; i += 64) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1024, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_t*)((char*)lds + dst_off), 16, (uint32_t)(lane * 16), 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < LDS_BYTES / 4; i += 64) out[i] = lds[i];
}

int main() {
  std::vector<uint32_t> h(256);
  for (int i = 0; i < 256; ++i) h[i] = 0x10000u + i;
  uint32_t *src, *out;
  if (hipMalloc(&src, 1024) != hipSuccess || hipMalloc(&out, LDS_BYTES) != hipSuccess) return 1;
  hipMemcpy(src, h.data(), 1024, hipMemcpyHostToDevice);
  const int offs[] = {0, 64 * 1024, 96 * 1024, 127 * 1024, 128 * 1024, 130 * 1024, 140 * 1024, 150 * 1024};
  std::vector<uint32_t> r(LDS_BYTES / 4);
  int bad = 0;
  for (int off : offs) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, off, out);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed at %d\n", off); return 1; }
    hipMemcpy(r.data(), out, LDS_BYTES, hipMemcpyDeviceToHost);
    bool at = true;
    for (int i = 0; i < 256; ++i) at &= r[off / 4 + i] == h[i];
    int landed = -1;
    for (int w = 0; w + 256 <= LDS_BYTES / 4 && landed < 0; w += 4) {
      if (r[w] != h[0]) continue;
      bool ok = true;
      for (int i = 0; i < 256 && ok; ++i) ok = r[w + i] == h[i];
      if (ok) landed = w * 4;
    }
    printf("dma to %6d B: %s (pattern found at %d)\n", off, at ? "landed" : "MISSING", landed);
    bad += !at;
  }
  printf("%s\n", bad ? "LDS-DMA does not reach every offset" : "LDS-DMA reaches every probed offset");
  return 0;
}
