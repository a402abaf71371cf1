// CRC-32C (Castagnoli) with TF/LevelDB "masking", used by the TFRecord event
// files (F23) and the TensorBundle checkpoint format (F21).  Slicing-by-8
// table implementation; SSE4.2 hardware path when available.
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

#define TDE_API extern "C" __attribute__((visibility("default")))

namespace {

uint32_t g_table[8][256];
bool g_init = false;

void init_tables() {
  const uint32_t poly = 0x82F63B78u;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xFF];
  g_init = true;
}

uint32_t extend_sw(uint32_t crc, const uint8_t* p, size_t n) {
  if (!g_init) init_tables();
  crc = ~crc;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = g_table[7][lo & 0xFF] ^ g_table[6][(lo >> 8) & 0xFF] ^ g_table[5][(lo >> 16) & 0xFF] ^
          g_table[4][lo >> 24] ^ g_table[3][hi & 0xFF] ^ g_table[2][(hi >> 8) & 0xFF] ^
          g_table[1][(hi >> 16) & 0xFF] ^ g_table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ g_table[0][(crc ^ *p++) & 0xFF];
  return ~crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t extend_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
#endif

bool has_sse42() {
#if defined(__x86_64__)
  return __builtin_cpu_supports("sse4.2");
#else
  return false;
#endif
}

}  // namespace

namespace tde_host {
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
#if defined(__x86_64__)
  static const bool hw = has_sse42();
  if (hw) return extend_hw(crc, (const uint8_t*)data, n);
#endif
  return extend_sw(crc, (const uint8_t*)data, n);
}
uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
uint32_t crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t crc32c_unmask(uint32_t m) {
  uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}
}  // namespace tde_host

TDE_API uint32_t tde_crc32c(const void* data, size_t n) { return tde_host::crc32c(data, n); }
TDE_API uint32_t tde_crc32c_extend(uint32_t crc, const void* data, size_t n) {
  return tde_host::crc32c_extend(crc, data, n);
}
TDE_API uint32_t tde_crc32c_masked(const void* data, size_t n) {
  return tde_host::crc32c_mask(tde_host::crc32c(data, n));
}
TDE_API uint32_t tde_crc32c_mask(uint32_t c) { return tde_host::crc32c_mask(c); }
TDE_API uint32_t tde_crc32c_unmask(uint32_t c) { return tde_host::crc32c_unmask(c); }
