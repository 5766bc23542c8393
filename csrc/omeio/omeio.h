// Native artifact I/O for the model agent and the engine's weight loader.
//
//  * safetensors header parsing (8-byte LE header length + JSON, bounded)          — agent + loader
//  * parallel pread -> pinned staging -> hipMemcpyAsync into HBM (double-buffered) — loader
//  * chunked parallel file copy with MD5 / byte verification                         — agent (gopher)
//  * AES-256-GCM file decryption (OpenSSL EVP)                                        — ome-agent enigma
//
// C ABI (ctypes) so Python never needs a build of its own.  All functions return 0 on success
// and a negative errno-style code otherwise; omeio_last_error() gives the message.
#pragma once
#include <cstddef>
#include <cstdint>

#define OMEIO_API extern "C" __attribute__((visibility("default")))

OMEIO_API const char* omeio_last_error();

// Reads the JSON header of a .safetensors file into `buf` (capacity `cap`, NUL-terminated).
// *header_len receives the JSON length, *data_offset the byte offset of the tensor data.
OMEIO_API int omeio_st_header(const char* path, char* buf, size_t cap, uint64_t* header_len,
                              uint64_t* data_offset);

// Copies `n` byte ranges of one file into device memory.  Ranges are split over `nthreads`
// reader threads, each owning two pinned staging buffers of `chunk` bytes so the pread of
// chunk i+1 overlaps the DMA of chunk i.  `stream` is a hipStream_t (0 = null stream); the
// call returns after all copies have completed.
OMEIO_API int omeio_load_ranges(const char* path, int n, const uint64_t* file_offsets, const uint64_t* sizes,
                                void* const* dst_device, void* stream, int nthreads, uint64_t chunk);

// Same, into host memory (no GPU needed) — used by CPU loads and tests.
OMEIO_API int omeio_read_ranges(const char* path, int n, const uint64_t* file_offsets, const uint64_t* sizes,
                                void* const* dst_host, int nthreads);

// Column shard of a row-major tensor: nrows slices of row_bytes starting at file_off with a
// file_stride between rows, packed contiguously into device memory (TP row-parallel weights:
// each rank reads and uploads only its 1/TP of every row).  omeio_read_strided: same, to host.
OMEIO_API int omeio_load_strided(const char* path, uint64_t file_off, uint64_t nrows, uint64_t file_stride,
                                 uint64_t row_bytes, void* dst_device, void* stream, int nthreads, uint64_t chunk);
OMEIO_API int omeio_read_strided(const char* path, uint64_t file_off, uint64_t nrows, uint64_t file_stride,
                                 uint64_t row_bytes, void* dst_host);
// Bytes pread by this process so far (loader statistics).
OMEIO_API uint64_t omeio_bytes_read();

// Parallel chunked copy src -> dst (creates/truncates dst).  If md5_hex (33 bytes) is non-null
// it receives the MD5 of the content.
OMEIO_API int omeio_copy_file(const char* src, const char* dst, int nthreads, char* md5_hex);

// MD5 of a file (hex, 33 bytes incl. NUL).
OMEIO_API int omeio_md5_file(const char* path, char* md5_hex);

// AES-256-GCM.  Layout of an encrypted file: 12-byte nonce | ciphertext | 16-byte tag.
OMEIO_API int omeio_aes_gcm_encrypt_file(const char* src, const char* dst, const uint8_t* key32,
                                         const uint8_t* nonce12);
OMEIO_API int omeio_aes_gcm_decrypt_file(const char* src, const char* dst, const uint8_t* key32);
// In-memory variants (the data-encryption key itself is wrapped this way).
OMEIO_API int omeio_aes_gcm_decrypt(const uint8_t* in, size_t in_len, const uint8_t* key32, uint8_t* out,
                                    size_t* out_len);
OMEIO_API int omeio_aes_gcm_encrypt(const uint8_t* in, size_t in_len, const uint8_t* key32, const uint8_t* nonce12,
                                    uint8_t* out, size_t* out_len);

// ---- Xet CAS chunk decoding (xet.cpp) -------------------------------------------------------
// A xorb byte range is a run of chunks, each an 8-byte header
//   [version u8][compressed length u24 LE][scheme u8][uncompressed length u24 LE]
// followed by its payload; scheme 0 = stored, 1 = LZ4 frame, 2 = byte-grouping-4 then LZ4 frame.
// omeio_xet_scan: number of chunks and total decoded size of `src` (validates the headers).
OMEIO_API int omeio_xet_scan(const uint8_t* src, size_t len, uint64_t* n_chunks, uint64_t* total);
// omeio_xet_decode: decodes every chunk into `dst` (capacity `cap`); offsets[i] / offsets[i + 1]
// bound chunk i in `dst` (`offsets` holds max_chunks + 1 entries).  Returns the chunk count.
OMEIO_API int64_t omeio_xet_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap, uint64_t* offsets,
                                   uint64_t max_chunks);
// raw LZ4 block / frame decoders (exposed for tests and other callers); return bytes written or < 0
OMEIO_API int64_t omeio_lz4_block_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap);
OMEIO_API int64_t omeio_lz4_frame_decode(const uint8_t* src, size_t len, uint8_t* dst, size_t cap);

int omeio_fail(int code, const char* msg);

// RSA PKCS#1 v1.5 / SHA-256 (OpenSSL: blinded constant-time signing, strict DigestInfo verify).
OMEIO_API int omeio_rsa_sign_sha256(const char* pem, size_t pem_len, const uint8_t* msg, size_t n, uint8_t* sig,
                                    size_t* sig_len);
OMEIO_API int omeio_rsa_verify_sha256(const char* pem, size_t pem_len, const uint8_t* msg, size_t n,
                                      const uint8_t* sig, size_t sig_len);
// Fresh RSA key pair: PKCS#8 private PEM + SubjectPublicKeyInfo public PEM.
OMEIO_API int omeio_rsa_keygen(int bits, char* priv_pem, size_t priv_cap, char* pub_pem, size_t pub_cap);
// X.509: RFC 2253 subject line and SHA-1 / SHA-256 DER fingerprints ("AA:BB:..."; 60 / 96 bytes).
OMEIO_API int omeio_x509_info(const char* pem, size_t n, char* subject, size_t subject_cap, char* sha1_fp,
                              char* sha256_fp);
