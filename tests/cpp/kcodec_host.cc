// Host build of cilium_amd/csrc/l7m_kcodec.h (TEST INFRASTRUCTURE): lets the
// CPU tests check the exact decoding / re-reading logic the GPU's second pass
// runs against the zlib-based oracle without a GPU.  Never used by the
// product (which runs l7m_kcodec.h only inside kafka_codec_kernel).
#include <cstdlib>
#include <vector>

#include "../../cilium_amd/csrc/l7m_kcodec.h"

extern "C" int kc_host_check(const uint8_t* val, uint32_t len, uint32_t codec, int32_t version, uint32_t slab_bytes) {
  static uint32_t tab[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    init = true;
  }
  std::vector<uint8_t> slab(slab_bytes);
  l7m::KcInflateScratch s;
  return l7m::kc_check_value(val, len, codec, static_cast<int16_t>(version), slab.data(), slab_bytes, tab, s);
}

// kc_check_produce on one whole ProduceReq record (what the GPU's second pass
// runs per queued request): 0 ok, 1 ReadRequest error, 2 unsupported.
extern "C" int kc_host_check_produce(const uint8_t* rec, uint32_t len, uint32_t slab_bytes) {
  static uint32_t tab[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    init = true;
  }
  std::vector<uint8_t> slab(slab_bytes);
  l7m::KcInflateScratch s;
  return l7m::kc_check_produce(rec, len, slab.data(), slab_bytes, tab, s);
}

// kc_unsnappy alone (framed or bare block): 0 decoded (*out_len bytes), 1
// error, 2 over cap.  For the snappy known-answer tests.
extern "C" int kc_host_unsnappy(const uint8_t* src, uint32_t n, uint8_t* out, uint32_t cap, uint32_t* out_len) {
  const int rc = l7m::kc_unsnappy(src, n, out, cap, cap, out_len);
  return rc == l7m::kCodecOk ? 0 : rc == l7m::kCodecErr ? 1 : 2;
}
