// AES-256-GCM (NIST SP 800-38D) on AES-NI + PCLMULQDQ for the EE envelope
// encryption (reference ee/pkg/encryption/aes_gcm.go; no crypto library is
// available in this image, so the primitive is native).  Counter mode with the
// 96-bit IV convention (J0 = IV || 0^31 || 1), GHASH via carry-less multiply on
// byte-reflected operands, constant-time tag comparison.
#include <immintrin.h>
#include <wmmintrin.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

struct Aes256 {
  __m128i rk[15];
};

inline __m128i expand_a(__m128i t1, __m128i t2) {
  t2 = _mm_shuffle_epi32(t2, 0xff);
  __m128i t4 = _mm_slli_si128(t1, 4);
  t1 = _mm_xor_si128(t1, t4);
  t4 = _mm_slli_si128(t4, 4);
  t1 = _mm_xor_si128(t1, t4);
  t4 = _mm_slli_si128(t4, 4);
  t1 = _mm_xor_si128(t1, t4);
  return _mm_xor_si128(t1, t2);
}

inline __m128i expand_b(__m128i t1, __m128i t3) {
  __m128i t2 = _mm_shuffle_epi32(_mm_aeskeygenassist_si128(t1, 0x0), 0xaa);
  __m128i t4 = _mm_slli_si128(t3, 4);
  t3 = _mm_xor_si128(t3, t4);
  t4 = _mm_slli_si128(t4, 4);
  t3 = _mm_xor_si128(t3, t4);
  t4 = _mm_slli_si128(t4, 4);
  t3 = _mm_xor_si128(t3, t4);
  return _mm_xor_si128(t3, t2);
}

#define OMNIA_KEYGEN(RC, I)                                   \
  t1 = expand_a(t1, _mm_aeskeygenassist_si128(t3, RC));        \
  k.rk[I] = t1;                                               \
  if (I + 1 < 15) {                                           \
    t3 = expand_b(t1, t3);                                    \
    k.rk[I + 1] = t3;                                         \
  }

void key_expand(const uint8_t* key, Aes256& k) {
  __m128i t1 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key));
  __m128i t3 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(key + 16));
  k.rk[0] = t1;
  k.rk[1] = t3;
  OMNIA_KEYGEN(0x01, 2)
  OMNIA_KEYGEN(0x02, 4)
  OMNIA_KEYGEN(0x04, 6)
  OMNIA_KEYGEN(0x08, 8)
  OMNIA_KEYGEN(0x10, 10)
  OMNIA_KEYGEN(0x20, 12)
  t1 = expand_a(t1, _mm_aeskeygenassist_si128(t3, 0x40));
  k.rk[14] = t1;
}
#undef OMNIA_KEYGEN

inline __m128i encrypt_block(const Aes256& k, __m128i x) {
  x = _mm_xor_si128(x, k.rk[0]);
  for (int i = 1; i < 14; ++i) x = _mm_aesenc_si128(x, k.rk[i]);
  return _mm_aesenclast_si128(x, k.rk[14]);
}

inline __m128i bswap128(__m128i x) {
  const __m128i m = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  return _mm_shuffle_epi8(x, m);
}

// GF(2^128) multiply of byte-reflected operands (Intel CLMUL white paper, Alg. 5)
inline __m128i gfmul(__m128i a, __m128i b) {
  __m128i t3 = _mm_clmulepi64_si128(a, b, 0x00);
  __m128i t4 = _mm_clmulepi64_si128(a, b, 0x10);
  __m128i t5 = _mm_clmulepi64_si128(a, b, 0x01);
  __m128i t6 = _mm_clmulepi64_si128(a, b, 0x11);
  t4 = _mm_xor_si128(t4, t5);
  t5 = _mm_slli_si128(t4, 8);
  t4 = _mm_srli_si128(t4, 8);
  t3 = _mm_xor_si128(t3, t5);
  t6 = _mm_xor_si128(t6, t4);
  __m128i t7 = _mm_srli_epi32(t3, 31);
  __m128i t8 = _mm_srli_epi32(t6, 31);
  t3 = _mm_slli_epi32(t3, 1);
  t6 = _mm_slli_epi32(t6, 1);
  __m128i t9 = _mm_srli_si128(t7, 12);
  t8 = _mm_slli_si128(t8, 4);
  t7 = _mm_slli_si128(t7, 4);
  t3 = _mm_or_si128(t3, t7);
  t6 = _mm_or_si128(t6, t8);
  t6 = _mm_or_si128(t6, t9);
  t7 = _mm_slli_epi32(t3, 31);
  t8 = _mm_slli_epi32(t3, 30);
  t9 = _mm_slli_epi32(t3, 25);
  t7 = _mm_xor_si128(t7, t8);
  t7 = _mm_xor_si128(t7, t9);
  t8 = _mm_srli_si128(t7, 4);
  t7 = _mm_slli_si128(t7, 12);
  t3 = _mm_xor_si128(t3, t7);
  __m128i t2 = _mm_srli_epi32(t3, 1);
  t4 = _mm_srli_epi32(t3, 2);
  t5 = _mm_srli_epi32(t3, 7);
  t2 = _mm_xor_si128(t2, t4);
  t2 = _mm_xor_si128(t2, t5);
  t2 = _mm_xor_si128(t2, t8);
  t3 = _mm_xor_si128(t3, t2);
  return _mm_xor_si128(t6, t3);
}

struct Ghash {
  __m128i h, y;
  explicit Ghash(__m128i h_) : h(h_), y(_mm_setzero_si128()) {}
  void update(const uint8_t* p, size_t n) {
    for (size_t o = 0; o < n; o += 16) {
      uint8_t blk[16] = {0};
      std::memcpy(blk, p + o, n - o < 16 ? n - o : 16);
      const __m128i x = bswap128(_mm_loadu_si128(reinterpret_cast<const __m128i*>(blk)));
      y = gfmul(_mm_xor_si128(y, x), h);
    }
  }
  __m128i finish(uint64_t aad_len, uint64_t ct_len) {
    const __m128i lens = _mm_set_epi64x((long long)(aad_len * 8), (long long)(ct_len * 8));
    y = gfmul(_mm_xor_si128(y, lens), h);
    return bswap128(y);
  }
};

inline __m128i inc32(__m128i ctr) {
  uint8_t b[16];
  _mm_storeu_si128(reinterpret_cast<__m128i*>(b), ctr);
  uint32_t c = ((uint32_t)b[12] << 24) | ((uint32_t)b[13] << 16) | ((uint32_t)b[14] << 8) | b[15];
  ++c;
  b[12] = c >> 24; b[13] = c >> 16; b[14] = c >> 8; b[15] = c;
  return _mm_loadu_si128(reinterpret_cast<const __m128i*>(b));
}

void ctr_xor(const Aes256& k, __m128i ctr, const uint8_t* in, uint8_t* out, size_t n) {
  size_t o = 0;
  for (; o + 16 <= n; o += 16) {
    ctr = inc32(ctr);
    const __m128i ks = encrypt_block(k, ctr);
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + o));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + o), _mm_xor_si128(x, ks));
  }
  if (o < n) {
    ctr = inc32(ctr);
    uint8_t ks[16];
    _mm_storeu_si128(reinterpret_cast<__m128i*>(ks), encrypt_block(k, ctr));
    for (size_t i = 0; o + i < n; ++i) out[o + i] = in[o + i] ^ ks[i];
  }
}

void check_cpu() {
  static const bool ok = __builtin_cpu_supports("aes") && __builtin_cpu_supports("pclmul") &&
                         __builtin_cpu_supports("ssse3");
  if (!ok) throw std::runtime_error("AES-NI / PCLMULQDQ not available on this CPU");
}

struct Ctx {
  Aes256 k;
  __m128i h, j0;
  Ctx(const std::string& key, const std::string& iv) {
    if (key.size() != 32) throw std::invalid_argument("AES-256-GCM needs a 32-byte key");
    if (iv.size() != 12) throw std::invalid_argument("AES-GCM nonce must be 12 bytes");
    check_cpu();
    key_expand(reinterpret_cast<const uint8_t*>(key.data()), k);
    h = bswap128(encrypt_block(k, _mm_setzero_si128()));
    uint8_t j[16] = {0};
    std::memcpy(j, iv.data(), 12);
    j[15] = 1;
    j0 = _mm_loadu_si128(reinterpret_cast<const __m128i*>(j));
  }
  __m128i tag(const std::string& aad, const uint8_t* ct, size_t n) {
    Ghash g(h);
    g.update(reinterpret_cast<const uint8_t*>(aad.data()), aad.size());
    g.update(ct, n);
    return _mm_xor_si128(g.finish(aad.size(), n), encrypt_block(k, j0));
  }
};

py::bytes encrypt(const std::string& key, const std::string& iv, const std::string& pt,
                  const std::string& aad) {
  std::string out(pt.size() + 16, '\0');
  {
    py::gil_scoped_release rel;
    Ctx c(key, iv);
    auto* o = reinterpret_cast<uint8_t*>(&out[0]);
    ctr_xor(c.k, c.j0, reinterpret_cast<const uint8_t*>(pt.data()), o, pt.size());
    _mm_storeu_si128(reinterpret_cast<__m128i*>(o + pt.size()), c.tag(aad, o, pt.size()));
  }
  return py::bytes(out);
}

py::bytes decrypt(const std::string& key, const std::string& iv, const std::string& data,
                  const std::string& aad) {
  if (data.size() < 16) throw std::invalid_argument("ciphertext shorter than the tag");
  const size_t n = data.size() - 16;
  std::string out(n, '\0');
  bool ok;
  {
    py::gil_scoped_release rel;
    Ctx c(key, iv);
    const auto* ct = reinterpret_cast<const uint8_t*>(data.data());
    uint8_t t[16];
    _mm_storeu_si128(reinterpret_cast<__m128i*>(t), c.tag(aad, ct, n));
    uint8_t diff = 0;
    for (int i = 0; i < 16; ++i) diff |= t[i] ^ ct[n + i];
    ok = diff == 0;
    if (ok) ctr_xor(c.k, c.j0, ct, reinterpret_cast<uint8_t*>(&out[0]), n);
  }
  if (!ok) throw py::value_error("AES-GCM authentication failed");
  return py::bytes(out);
}

}  // namespace

void register_aes_gcm(py::module_& m) {
  m.def("aes_gcm_encrypt", &encrypt, py::arg("key"), py::arg("iv"), py::arg("plaintext"),
        py::arg("aad") = std::string(), "AES-256-GCM encrypt -> ciphertext || 16-byte tag");
  m.def("aes_gcm_decrypt", &decrypt, py::arg("key"), py::arg("iv"), py::arg("data"),
        py::arg("aad") = std::string(), "AES-256-GCM decrypt (raises ValueError on bad tag)");
}
