// featurize.cpp — host-side chunker and hashed bag-of-words features (C ABI in include/rfx.h).
//
// The reference forwards chunking to Gemini (chunking_config, gemini_rag.py:324-326) and has
// exactly one tokeniser of its own: scripts/benchmark/metrics.py:13-19 (_normalize):
//     text.lower(); re.sub(r"[^a-z0-9\s]", " ", text); split(); drop {"a", "an", "the"}.
// Restated on UTF-8 bytes: after lower-casing, a token character is an ASCII [a-z0-9] byte and
// every other byte separates tokens (all non-ASCII UTF-8 bytes are >= 0x80, so this is exact
// once the caller has applied str.lower(); ASCII A-Z are lower-cased here).
//
// Chunking follows Gemini's white_space_config: windows of max_tokens whitespace-delimited
// tokens, consecutive windows sharing `overlap` tokens.  Whitespace = the ASCII bytes that
// Python's bytes.split() treats as whitespace: \t \n \v \f \r and space, plus \x1c-\x1f.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rfx.h"

namespace {

inline bool is_ws(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 28 && c <= 31); }

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

inline uint64_t fnv1a64(const unsigned char* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

}  // namespace

extern "C" {

int rfx_chunk_whitespace(const char* text, int64_t len, int max_tokens, int overlap, int64_t* out_spans_h,
                         int64_t cap, int64_t* out_n) {
  if (!out_n || len < 0 || (len > 0 && !text)) return RFX_EINVAL;
  if (max_tokens < 1 || max_tokens > 65536 || overlap < 0 || overlap >= max_tokens) return RFX_EINVAL;
  const unsigned char* t = (const unsigned char*)text;
  std::vector<std::pair<int64_t, int64_t>> toks;
  int64_t i = 0;
  while (i < len) {
    while (i < len && is_ws(t[i])) ++i;
    if (i >= len) break;
    const int64_t s = i;
    while (i < len && !is_ws(t[i])) ++i;
    toks.emplace_back(s, i);
  }
  int64_t n = 0;
  const int64_t nt = (int64_t)toks.size();
  int64_t start = 0;
  while (nt > 0) {
    const int64_t end = std::min<int64_t>(start + max_tokens, nt);
    if (n < cap && out_spans_h) {
      out_spans_h[2 * n] = toks[(size_t)start].first;
      out_spans_h[2 * n + 1] = toks[(size_t)end - 1].second;
    }
    ++n;
    if (end == nt) break;
    start = end - overlap;
  }
  *out_n = n;
  return RFX_OK;
}

int rfx_featurize(const char* text, const int64_t* spans_h, int64_t n, int V, uint64_t hash_seed,
                  int32_t* indptr_h, int32_t* bucket_h, int16_t* count_h, int64_t cap_nnz, int64_t* out_nnz) {
  if (!out_nnz || n < 0 || (n > 0 && (!text || !spans_h || !indptr_h))) return RFX_EINVAL;
  if (V < 16 || (V & (V - 1))) return RFX_EINVAL;
  const unsigned char* t = (const unsigned char*)text;
  int64_t nnz = 0;
  std::vector<std::pair<int32_t, int32_t>> acc;  // (bucket, signed count)
  std::string tok;
  indptr_h[0] = 0;
  for (int64_t c = 0; c < n; ++c) {
    const int64_t b = spans_h[2 * c], e = spans_h[2 * c + 1];
    if (b < 0 || e < b) return RFX_EINVAL;
    acc.clear();
    int64_t i = b;
    // at most 65536 normalised tokens per chunk: keeps every f32 partial sum of the MFMA
    // embedding below 2^24 quanta, i.e. exact (k_embed.hip).
    while (i < e && (int64_t)acc.size() < 65536) {
      // skip separators
      while (i < e) {
        unsigned char ch = t[i];
        if (ch >= 'A' && ch <= 'Z') ch = (unsigned char)(ch - 'A' + 'a');
        if ((ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9')) break;
        ++i;
      }
      if (i >= e) break;
      tok.clear();
      while (i < e) {
        unsigned char ch = t[i];
        if (ch >= 'A' && ch <= 'Z') ch = (unsigned char)(ch - 'A' + 'a');
        if (!((ch >= 'a' && ch <= 'z') || (ch >= '0' && ch <= '9'))) break;
        tok.push_back((char)ch);
        ++i;
      }
      if (tok == "a" || tok == "an" || tok == "the") continue;
      const uint64_t h = splitmix64(fnv1a64((const unsigned char*)tok.data(), tok.size()) + hash_seed);
      const int32_t bucket = (int32_t)(h & (uint64_t)(V - 1));
      const int32_t sign = (h >> 63) ? -1 : 1;
      acc.emplace_back(bucket, sign);
    }
    std::sort(acc.begin(), acc.end());
    size_t j = 0;
    while (j < acc.size()) {
      const int32_t bk = acc[j].first;
      int32_t s = 0;
      while (j < acc.size() && acc[j].first == bk) s += acc[j++].second;
      if (s == 0) continue;
      s = std::max(-256, std::min(256, s));
      if (nnz < cap_nnz && bucket_h && count_h) {
        bucket_h[nnz] = bk;
        count_h[nnz] = (int16_t)s;
      }
      ++nnz;
    }
    indptr_h[c + 1] = (int32_t)std::min<int64_t>(nnz, INT32_MAX);
  }
  *out_nnz = nnz;
  return RFX_OK;
}

}  // extern "C"
