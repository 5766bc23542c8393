// Same-node KV-page transport for prefill/decode disaggregation (SURVEY.md §2.7 PD row, §2.8
// "Mooncake transfer engine" -> MI355X mapping, §5.8): the decode engine exports its paged KV
// tensors through hipIpc handles once; the prefill engine maps them and writes the prompt's pages
// straight into the decode GPU's HBM over xGMI with a copy kernel running on the PREFILL GPU
// (remote stores, no host bounce, no CU time on the decode GPU while it keeps decoding).
//
// The reference moves these bytes with Mooncake over RDMA NICs (config/runtimes/srt/
// deepseek-rdma-pd-rt.yaml:79-80); on one 8x MI355X node every GPU pair has a direct xGMI link.
//
// Page images are opaque bytes here (bf16 or fp8 caches, K [P, D] or transposed V [D, P] per
// kv head): a "page" of a layer is `page_bytes` contiguous bytes at `page * page_stride`.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#define OME_API extern "C" __attribute__((visibility("default")))

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// base-relative export: the caching allocator sub-allocates, so ship (handle of the owning
// allocation, byte offset of the tensor inside it)
OME_API int ome_kvlink_export(const void* ptr, void* handle_out, int64_t* offset_out) {
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr));
  if (e != hipSuccess) return (int)e;
  e = hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle_out), base);
  if (e != hipSuccess) return (int)e;
  *offset_out = (int64_t)((const char*)ptr - (const char*)base);
  return 0;
}

OME_API int ome_kvlink_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// map a peer allocation into this process (peer access enabled lazily for every local device)
OME_API int ome_kvlink_open(const void* handle, void** base_out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  hipError_t e = hipIpcOpenMemHandle(base_out, h, hipIpcMemLazyEnablePeerAccess);
  return (int)e;
}

OME_API int ome_kvlink_close(void* base) { return (int)hipIpcCloseMemHandle(base); }

// One workgroup per (page pair, layer tensor): 16-byte vector copies of one page image from a
// local tensor to a (peer-mapped) destination tensor.  `src_bases` / `dst_bases` hold one base
// pointer per layer tensor (K and V of every layer = 2L tensors).
__global__ __launch_bounds__(256) void kvlink_copy_kernel(const char* const* __restrict__ src_bases,
                                                          char* const* __restrict__ dst_bases,
                                                          const int* __restrict__ src_pages,
                                                          const int* __restrict__ dst_pages, int n_pages,
                                                          int64_t page_stride, int64_t page_bytes) {
  const int p = blockIdx.x, t = blockIdx.y;
  if (p >= n_pages) return;
  const u32x4* src = reinterpret_cast<const u32x4*>(src_bases[t] + (int64_t)src_pages[p] * page_stride);
  u32x4* dst = reinterpret_cast<u32x4*>(dst_bases[t] + (int64_t)dst_pages[p] * page_stride);
  const int64_t n16 = page_bytes / 16;
  for (int64_t i = threadIdx.x; i < n16; i += blockDim.x) {
    // non-temporal: the destination is another GPU's HBM; do not keep the lines in our L2
    __builtin_nontemporal_store(src[i], dst + i);
  }
}

// src_bases / dst_bases / src_pages / dst_pages are DEVICE arrays (staged by the caller).
OME_API int ome_kvlink_copy(const void* src_bases, const void* dst_bases, const int* src_pages, const int* dst_pages,
                            int n_pages, int n_tensors, int64_t page_stride, int64_t page_bytes,
                            hipStream_t stream) {
  if (n_pages <= 0 || n_tensors <= 0) return 0;
  if (page_bytes % 16 != 0 || page_stride % 16 != 0) return -2;
  dim3 grid(n_pages, n_tensors);
  kvlink_copy_kernel<<<grid, 256, 0, stream>>>((const char* const*)src_bases, (char* const*)dst_bases, src_pages,
                                              dst_pages, n_pages, page_stride, page_bytes);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
