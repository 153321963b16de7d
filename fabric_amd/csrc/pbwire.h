// pbwire.h -- protobuf wire decoding with the semantics of google.golang.org/protobuf
// v1.33.0 (vendored by the reference, go.mod:42) for the proto3 Fabric messages on the
// committer path.  Host-side, allocation-free, single pass:
//   * tag varint; field number outside [1, 2^29-1] -> error; END_GROUP at message level -> error
//   * varint <= 10 bytes, 10th byte <= 1
//   * wire types 6/7 -> error; unknown START_GROUP skipped to its matching END_GROUP
//   * known field with the wrong wire type -> skipped as unknown (errUnknown path)
//   * `string` -> must be valid UTF-8 (Go utf8.Valid) else error
//   * `bytes` -> last occurrence wins; empty decodes to nil (consumeBytesNoZero)
//   * singular embedded message: every occurrence is recorded and decoded in order into the
//     same value (merge); repeated fields append
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace pbw {

struct Span {
  const uint8_t *p = nullptr;
  uint32_t n = 0;
  bool nil() const { return n == 0; }  // proto3 bytes: present <=> non-empty
  std::string str() const { return std::string(reinterpret_cast<const char *>(p), n); }
  bool eq(const char *s, size_t l) const { return n == l && (l == 0 || memcmp(p, s, l) == 0); }
  bool eq(const Span &o) const { return n == o.n && (n == 0 || memcmp(p, o.p, n) == 0); }
  // byte-lexicographic order (Go string comparison)
  bool operator<(const Span &o) const {
    const int c = memcmp(p, o.p, n < o.n ? n : o.n);
    return c < 0 || (c == 0 && n < o.n);
  }
};

inline bool rd_varint(const uint8_t *&p, const uint8_t *e, uint64_t &v) {
  v = 0;
  for (int i = 0; i < 10; i++) {
    if (p >= e) return false;
    const uint8_t c = *p++;
    if (i == 9 && c > 1) return false;
    v |= (uint64_t)(c & 0x7f) << (7 * i);
    if (c < 0x80) return true;
  }
  return false;
}

inline bool skip_value(const uint8_t *&p, const uint8_t *e, uint32_t num, int wt, int depth = 0) {
  uint64_t v;
  switch (wt) {
    case 0: return rd_varint(p, e, v);
    case 1: if (e - p < 8) return false; p += 8; return true;
    case 5: if (e - p < 4) return false; p += 4; return true;
    case 2:
      if (!rd_varint(p, e, v) || v > (uint64_t)(e - p)) return false;
      p += v;
      return true;
    case 3:
      if (depth > 10000) return false;
      for (;;) {
        uint64_t tag;
        if (!rd_varint(p, e, tag)) return false;
        const uint64_t n2 = tag >> 3;
        const int w2 = (int)(tag & 7);
        if (n2 < 1 || n2 > (1u << 29) - 1) return false;
        if (w2 == 4) return n2 == num;
        if (!skip_value(p, e, (uint32_t)n2, w2, depth + 1)) return false;
      }
    default: return false;  // END_GROUP without START, or 6/7
  }
}

// Go utf8.Valid
inline bool utf8_valid(const uint8_t *s, size_t n) {
  size_t i = 0;
  while (i + 8 <= n) {  // ASCII fast path
    uint64_t w;
    memcpy(&w, s + i, 8);
    if (w & 0x8080808080808080ull) break;
    i += 8;
  }
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    size_t len;
    uint32_t cp;
    if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
    else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
    else return false;
    if (i + len > n) return false;
    for (size_t k = 1; k < len; k++) {
      const uint8_t d = s[i + k];
      if ((d & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (d & 0x3F);
    }
    if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000)) return false;
    if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
    i += len;
  }
  return true;
}

enum Kind : uint8_t { K_NONE = 0, K_VARINT, K_BYTES, K_STRING, K_MSG, K_REP_MSG, K_REP_BYTES };

// Field visitor: returns the Kind for field number `num` (K_NONE = unknown) and receives
// decoded values.  decode() applies the wire rules and calls on_varint / on_len.
template <class V>
inline bool decode(const uint8_t *p, size_t n, V &vis) {
  const uint8_t *e = p + n;
  while (p < e) {
    uint64_t tag;
    if (!rd_varint(p, e, tag)) return false;
    const uint64_t num = tag >> 3;
    const int wt = (int)(tag & 7);
    if (num < 1 || num > (1u << 29) - 1) return false;
    if (wt == 4) return false;
    const Kind k = vis.kind((uint32_t)num);
    const int want = (k == K_VARINT) ? 0 : 2;
    if (k == K_NONE || wt != want) {
      if (!skip_value(p, e, (uint32_t)num, wt)) return false;
      continue;
    }
    if (k == K_VARINT) {
      uint64_t v;
      if (!rd_varint(p, e, v)) return false;
      vis.on_varint((uint32_t)num, v);
      continue;
    }
    uint64_t l;
    if (!rd_varint(p, e, l) || l > (uint64_t)(e - p)) return false;
    Span s{p, (uint32_t)l};
    p += l;
    if (k == K_STRING && !utf8_valid(s.p, s.n)) return false;
    if (!vis.on_len((uint32_t)num, s)) return false;
  }
  return true;
}

// A singular embedded message field: every occurrence, decoded in order = merge.
struct MsgField {
  bool present = false;
  Span first;                 // common case: one occurrence
  std::vector<Span> more;     // rare: further occurrences
  void add(Span s) {
    if (!present) { present = true; first = s; }
    else more.push_back(s);
  }
  template <class V> bool decode_into(V &vis) const {
    if (!present) return true;
    if (!pbw::decode(first.p, first.n, vis)) return false;
    for (const Span &s : more)
      if (!pbw::decode(s.p, s.n, vis)) return false;
    return true;
  }
};

inline int32_t as_int32(uint64_t v) { return (int32_t)(uint32_t)v; }

// Repeated field storage with N inline elements: the per-transaction decode allocates nothing
// in the common shapes (1 action, a handful of endorsements / namespaces).
template <class T, size_t N>
struct SmallVec {
  T inl[N];
  std::vector<T> heap;
  uint32_t cnt = 0;
  bool spilled = false;
  void push_back(const T &x) {
    if (!spilled) {
      if (cnt < N) { inl[cnt++] = x; return; }
      heap.assign(inl, inl + N);
      spilled = true;
    }
    heap.push_back(x);
    cnt++;
  }
  void clear() { cnt = 0; spilled = false; heap.clear(); }
  size_t size() const { return cnt; }
  bool empty() const { return cnt == 0; }
  T *data() { return spilled ? heap.data() : inl; }
  const T *data() const { return spilled ? heap.data() : inl; }
  T &operator[](size_t i) { return data()[i]; }
  const T &operator[](size_t i) const { return data()[i]; }
  T *begin() { return data(); }
  T *end() { return data() + cnt; }
  const T *begin() const { return data(); }
  const T *end() const { return data() + cnt; }
};

}  // namespace pbw
