// pbwire_dev.h -- protobuf wire decoding for device code (gfx950), the rules of pbwire.h
// (google.golang.org/protobuf v1.33.0 as vendored by the reference, go.mod:42) restated with
// fixed capacities: a capacity overflow sets `ovf` (the caller redoes the batch on the host or
// reports it) instead of allocating.  Shared by the committer kernels (blockdev.hip) and the
// MVCC kernels (mvcc.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blockdev.h"

namespace pbd {

#define DEV __device__ __forceinline__

// ------------------------------------------------------------------ protobuf wire (device)
struct S {  // absolute device span
  const uint8_t *p;
  uint32_t n;
};

// Message bytes are read a word at a time where the rules allow it: these kernels are bound by
// chains of dependent loads (one lane walks one transaction), not by bandwidth, so reading 4 or
// 16 bytes per load shortens the chains.  ld4: the 4 bytes at p (any alignment, little-endian)
// from the two aligned dwords covering them -- independent loads.  Over-read contract: up to 7
// bytes past a span's end (block arenas and the channel image carry >= 64 B of tail padding).
DEV uint32_t ld4(const uint8_t *p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}
DEV uint32_t lo_mask(uint32_t r) { return r >= 4u ? 0xFFFFFFFFu : ((1u << (8u * r)) - 1u); }

// Issue one load per 128-byte line of [p, p + n) -- independent loads, all in flight at once --
// so that a walk of the span that follows (one dependent load after another) finds its lines in
// the caches instead of paying the HBM latency at every field.  The loaded words are consumed by
// an empty asm (the loads are otherwise dead).
DEV void touch_lines(const uint8_t *p, uint32_t n) {
  const uintptr_t a0 = reinterpret_cast<uintptr_t>(p) & ~(uintptr_t)127;
  const uintptr_t a1 = reinterpret_cast<uintptr_t>(p) + n;
  uint32_t acc = 0;
  uintptr_t a = a0;
  for (; a + 8 * 128 <= a1; a += 8 * 128) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = *reinterpret_cast<const uint32_t *>(a + 128 * k);
#pragma unroll
    for (int k = 0; k < 8; k++) acc ^= v[k];
  }
  for (; a < a1; a += 128) acc ^= *reinterpret_cast<const uint32_t *>(a);
  asm volatile("" ::"v"(acc));
}

DEV bool s_eq(S a, S b) {
  if (a.n != b.n) return false;
  for (uint32_t i = 0; i < a.n; i += 4)
    if ((ld4(a.p + i) ^ ld4(b.p + i)) & lo_mask(a.n - i)) return false;
  return true;
}
DEV bool s_lt(S a, S b) {  // byte-lexicographic (Go string order): big-endian word compares
  const uint32_t m = a.n < b.n ? a.n : b.n;
  for (uint32_t i = 0; i < m; i += 4) {
    const uint32_t k = lo_mask(m - i);
    const uint32_t x = __builtin_bswap32(ld4(a.p + i) & k), y = __builtin_bswap32(ld4(b.p + i) & k);
    if (x != y) return x < y;
  }
  return a.n < b.n;
}

enum Kind : uint8_t { K_NONE = 0, K_VARINT, K_BYTES, K_STRING, K_MSG, K_REP_MSG, K_REP_BYTES };

DEV bool rd_varint(const uint8_t *&p, const uint8_t *e, uint64_t &v) {
  v = 0;
  int i = 0;
  if (e - p >= 4) {  // the first 4 bytes in one read (tags and lengths are 1-3 bytes)
    const uint32_t w = ld4(p);
    const uint32_t stop = ~w & 0x80808080u;  // bit 7 of byte k clear: the varint ends at k
    if (stop) {
      const uint32_t k = (uint32_t)__builtin_ctz(stop) >> 3;  // 0..3
      const uint32_t b0 = w & 0x7Fu, b1 = (w >> 8) & 0x7Fu, b2 = (w >> 16) & 0x7Fu, b3 = (w >> 24) & 0x7Fu;
      v = k == 0 ? b0 : k == 1 ? (b0 | b1 << 7) : k == 2 ? (b0 | b1 << 7 | b2 << 14) : (b0 | b1 << 7 | b2 << 14 | b3 << 21);
      p += k + 1;
      return true;
    }
    v = (w & 0x7Fu) | ((w >> 8) & 0x7Fu) << 7 | ((w >> 16) & 0x7Fu) << 14 | (uint64_t)((w >> 24) & 0x7Fu) << 21;
    p += 4;
    i = 4;
  }
  for (; i < 10; i++) {
    if (p >= e) return false;
    const uint8_t c = *p++;
    if (i == 9 && c > 1) return false;
    v |= (uint64_t)(c & 0x7f) << (7 * i);
    if (c < 0x80) return true;
  }
  return false;
}

// skip one field value (wire type wt of field num); START_GROUP nesting tracked on a small
// explicit stack (pbwire.h recurses; deeper than BD_MAX_GROUP -> overflow)
DEV bool skip_value(const uint8_t *&p, const uint8_t *e, uint32_t num, int wt, bool &ovf) {
  uint64_t v;
  switch (wt) {
    case 0: return rd_varint(p, e, v);
    case 1: if (e - p < 8) return false; p += 8; return true;
    case 5: if (e - p < 4) return false; p += 4; return true;
    case 2:
      if (!rd_varint(p, e, v) || v > (uint64_t)(e - p)) return false;
      p += v;
      return true;
    case 3: {
      uint32_t stack[BD_MAX_GROUP];
      int sp = 0;
      stack[sp++] = num;
      while (sp > 0) {
        uint64_t tag;
        if (!rd_varint(p, e, tag)) return false;
        const uint64_t n2 = tag >> 3;
        const int w2 = (int)(tag & 7);
        if (n2 < 1 || n2 > (1u << 29) - 1) return false;
        if (w2 == 4) {
          if (n2 != stack[sp - 1]) return false;
          sp--;
          continue;
        }
        if (w2 == 3) {
          if (sp == BD_MAX_GROUP) { ovf = true; return false; }
          stack[sp++] = (uint32_t)n2;
          continue;
        }
        if (w2 == 0) { if (!rd_varint(p, e, v)) return false; }
        else if (w2 == 1) { if (e - p < 8) return false; p += 8; }
        else if (w2 == 5) { if (e - p < 4) return false; p += 4; }
        else if (w2 == 2) { if (!rd_varint(p, e, v) || v > (uint64_t)(e - p)) return false; p += v; }
        else return false;
      }
      return true;
    }
    default: return false;
  }
}

DEV bool utf8_valid(const uint8_t *s, uint32_t n) {  // Go utf8.Valid
  uint32_t i = 0;
  while (i < n) {
    if (n - i >= 16) {  // ASCII runs 16 bytes per step (5 aligned dword loads)
      const uint32_t w = ld4(s + i) | ld4(s + i + 4) | ld4(s + i + 8) | ld4(s + i + 12);
      if (!(w & 0x80808080u)) { i += 16; continue; }
    } else if (n - i >= 4 && !(ld4(s + i) & 0x80808080u)) {
      i += 4;
      continue;
    }
    const uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t len, cp;
    if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
    else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
    else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
    else return false;
    if (i + len > n) return false;
    for (uint32_t k = 1; k < len; k++) {
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

// decode (pbwire.h decode): visitor kind / on_varint / on_len; ovf = a device capacity was hit
template <class V>
DEV bool decode(const uint8_t *p, uint32_t n, V &vis, bool &ovf) {
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
      if (!skip_value(p, e, (uint32_t)num, wt, ovf)) return false;
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
    S s{p, (uint32_t)l};
    p += l;
    if (k == K_STRING && !utf8_valid(s.p, s.n)) return false;
    if (!vis.on_len((uint32_t)num, s, ovf)) return false;
  }
  return true;
}
template <class V>
DEV bool decode(S s, V &vis, bool &ovf) { return decode(s.p, s.n, vis, ovf); }

DEV int32_t as_int32(uint64_t v) { return (int32_t)(uint32_t)v; }

// ------------------------------------------------------------------ visitors (device)
// Same field maps as fgv_visitors.h.  A singular embedded message field decodes every
// occurrence in order into one value (protobuf merge): visitors decode at on_len time.
struct VTwoBytes {  // Envelope / Header / SignatureHeader / TransactionAction / Endorsement / Prp
  S a{nullptr, 0}, b{nullptr, 0};
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) { (n == 1 ? a : b) = s; return true; }
};
struct VTimestamp {
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_VARINT : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VPayload {
  bool has_header = false;
  VTwoBytes hdr;  // channel_header, signature_header (all occurrences merged)
  S data{nullptr, 0};
  DEV Kind kind(uint32_t n) { return n == 1 ? K_MSG : n == 2 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 2) { data = s; return true; }
    has_header = true;
    return decode(s, hdr, ovf);
  }
};
struct VChannelHeader {
  int32_t type = 0;
  uint64_t epoch = 0;
  S channel_id{nullptr, 0}, tx_id{nullptr, 0}, extension{nullptr, 0};
  DEV Kind kind(uint32_t n) {
    switch (n) {
      case 1: case 2: case 6: return K_VARINT;
      case 3: return K_MSG;
      case 4: case 5: return K_STRING;
      case 7: case 8: return K_BYTES;
      default: return K_NONE;
    }
  }
  DEV void on_varint(uint32_t n, uint64_t v) {
    if (n == 1) type = as_int32(v);
    else if (n == 6) epoch = v;
  }
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 3) { VTimestamp t; return decode(s, t, ovf); }
    if (n == 4) channel_id = s;
    else if (n == 5) tx_id = s;
    else if (n == 7) extension = s;
    return true;
  }
};
struct VTransaction {  // repeated TransactionAction: count + the first
  uint32_t nact = 0;
  VTwoBytes first;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) {
    VTwoBytes a;
    if (!decode(s, a, ovf)) return false;
    if (nact == 0) first = a;
    nact++;
    return true;
  }
};
struct VEndorsedAction {
  S prp{nullptr, 0};
  uint32_t nend = 0;
  S ser[BD_MAX_END], sig[BD_MAX_END];
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_REP_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { prp = s; return true; }
    VTwoBytes e;
    if (!decode(s, e, ovf)) return false;
    if (nend == BD_MAX_END) { ovf = true; return false; }
    ser[nend] = e.a;
    sig[nend] = e.b;
    nend++;
    return true;
  }
};
struct VCcActionPayload {
  S ccpp{nullptr, 0};
  bool has_action = false;
  VEndorsedAction action;
  DEV Kind kind(uint32_t n) { return n == 1 ? K_BYTES : n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { ccpp = s; return true; }
    has_action = true;
    return decode(s, action, ovf);
  }
};
struct VChaincodeID {
  S path{nullptr, 0}, name{nullptr, 0}, version{nullptr, 0};
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? K_STRING : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) { (n == 1 ? path : n == 2 ? name : version) = s; return true; }
};
struct VResponse {
  DEV Kind kind(uint32_t n) { return n == 1 ? K_VARINT : n == 2 ? K_STRING : n == 3 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S, bool &) { return true; }
};
struct VCcAction {
  S results{nullptr, 0}, events{nullptr, 0};
  bool has_ccid = false;
  VChaincodeID ccid;
  DEV Kind kind(uint32_t n) { return (n == 1 || n == 2) ? K_BYTES : (n == 3 || n == 4) ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &ovf) {
    if (n == 1) { results = s; return true; }
    if (n == 2) { events = s; return true; }
    if (n == 3) { VResponse r; return decode(s, r, ovf); }
    has_ccid = true;
    return decode(s, ccid, ovf);
  }
};
struct VHdrExt {
  bool has_ccid = false;
  VChaincodeID ccid;
  DEV Kind kind(uint32_t n) { return n == 2 ? K_MSG : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t, S s, bool &ovf) { has_ccid = true; return decode(s, ccid, ovf); }
};
struct VCcEvent {
  S chaincode_id{nullptr, 0};
  DEV Kind kind(uint32_t n) { return (n >= 1 && n <= 3) ? K_STRING : n == 4 ? K_BYTES : K_NONE; }
  DEV void on_varint(uint32_t, uint64_t) {}
  DEV bool on_len(uint32_t n, S s, bool &) { if (n == 1) chaincode_id = s; return true; }
};
}  // namespace pbd
