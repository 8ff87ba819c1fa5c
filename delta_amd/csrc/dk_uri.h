// Reconciliation key of one file action, shared by host and device:
//   (java.net.URI(path), Optional<dvUniqueId>)   — LogReplayUtils.java:36-51,83-89 (kernel-api
//   internal/replay), DeletionVectorDescriptor.getUniqueId (internal/actions/
//   DeletionVectorDescriptor.java:167-174).
//
// Instead of materialising a URI object per row, each path is parsed once (JDK Parser grammar,
// RFC 2396 + RFC 2732 deviations) and emitted as a CANONICAL BYTE STREAM such that two paths give
// equal streams iff URI.equals holds:
//   scheme lower-cased; server-based host lower-cased; port as an integer; the two chars after
//   every '%' lower-cased (URI.equal()); a null component (no authority/query/fragment) is
//   distinguished from an empty one by a tag byte. Tag bytes are control bytes, which never occur
//   inside a parsed URI, so the stream is injective.
// The same emitter drives three sinks: a 64-bit hash (probe), a streaming comparator (exact
// verification of hash candidates) and a writer (JSON-tail keys).
//
// The common Delta path — a relative path of plain path characters with no ':', '%', '?', '#'
// and no leading "//" — is a pure pass-through: stream = TAG_PATH + raw bytes, hashed 8 B/step.
#pragma once
#include <stdint.h>
#include "dk_thrift.h"

namespace dk {

enum : uint8_t { TAG_SCHEME = 1, TAG_OPAQUE = 2, TAG_SERVER = 3, TAG_USERINFO = 4, TAG_HOST = 5,
                 TAG_PORT = 6, TAG_REGISTRY = 7, TAG_PATH = 8, TAG_QUERY = 9, TAG_FRAGMENT = 10 };

// ASCII char-class bits (RFC 2396 as used by java.net.URI)
enum : uint16_t {
  CC_DIGIT = 1, CC_ALPHA = 2, CC_HEX = 4, CC_MARK = 8, CC_RESERVED = 16,
  CC_PATHX = 32,      // ":@&=+$,;/"   extra pchar/path chars
  CC_USERX = 64,      // ";:&=+$,"     extra userinfo chars
  CC_REGX = 128,      // "$,;:@&=+"    extra reg_name chars
  CC_SERVX = 256,     // ".:@[]"       extra server chars
  CC_SIMPLE = 512,    // fast-path path chars: unreserved + "@&=+$,;/" (no ':' '%' '?' '#')
};

DK_HD uint16_t uri_class(uint8_t c) {
  uint16_t r = 0;
  if (c >= '0' && c <= '9') r |= CC_DIGIT | CC_HEX;
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) r |= CC_ALPHA;
  if ((c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F')) r |= CC_HEX;
  switch (c) {
    case '-': case '_': case '.': case '!': case '~': case '*': case '\'': case '(': case ')': r |= CC_MARK; break;
    default: break;
  }
  switch (c) { case ';': case '/': case '?': case ':': case '@': case '&': case '=': case '+': case '$': case ',': case '[': case ']': r |= CC_RESERVED; break; default: break; }
  switch (c) { case ':': case '@': case '&': case '=': case '+': case '$': case ',': case ';': case '/': r |= CC_PATHX; break; default: break; }
  switch (c) { case ';': case ':': case '&': case '=': case '+': case '$': case ',': r |= CC_USERX; break; default: break; }
  switch (c) { case '$': case ',': case ';': case ':': case '@': case '&': case '=': case '+': r |= CC_REGX; break; default: break; }
  switch (c) { case '.': case ':': case '@': case '[': case ']': r |= CC_SERVX; break; default: break; }
  if ((r & (CC_DIGIT | CC_ALPHA | CC_MARK)) || c == '@' || c == '&' || c == '=' || c == '+' || c == '$' ||
      c == ',' || c == ';' || c == '/')
    r |= CC_SIMPLE;
  return r;
}
DK_HD bool cc_unres(uint16_t k) { return (k & (CC_DIGIT | CC_ALPHA | CC_MARK)) != 0; }

DK_HD uint64_t kHashSeed(uint32_t seed) { return 0x243F6A8885A308D3ull * (uint64_t)(seed + 1); }

// ---- 64-bit streaming hash of a canonical stream ----
// The stream's first byte (always a TAG_* byte) is absorbed on its own, then the remaining bytes
// as 8-byte little-endian words, so for a plain relative path (stream = TAG_PATH + raw bytes) the
// words are exactly the raw 8-byte words of the path. One 64-bit multiply per word.
struct Hash64 {
  uint64_t h, buf;
  int nb, started;
  DK_HD void init(uint64_t seed) { h = seed ^ 0x9E3779B97F4A7C15ull; buf = 0; nb = 0; started = 0; }
  DK_HD static uint64_t mixw(uint64_t h, uint64_t w) {
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 29);
  }
  DK_HD void word(uint64_t w) { h = mixw(h, w); }
  DK_HD void put(uint8_t b) {
    if (!started) { started = 1; h = mixw(h, 0x100u | b); return; }
    buf |= (uint64_t)b << (8 * nb);
    if (++nb == 8) { word(buf); buf = 0; nb = 0; }
  }
  DK_HD static uint64_t fin(uint64_t h, uint64_t tail, uint64_t total_len) {
    uint64_t x = mixw(mixw(h, tail), total_len);
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x ? x : 1;   // 0 marks an empty table slot / "not computed"
  }
  DK_HD uint64_t final_(uint64_t total_len) { return fin(h, buf, total_len); }
};

DK_HD uint64_t hash_combine(uint64_t a, uint64_t b) {
  uint64_t x = a ^ (b + 0x9E3779B97F4A7C15ull + (a << 6) + (a >> 2));
  x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33;
  return x ? x : 1;
}

// ---- sinks ----
struct HashSink {
  Hash64 hs; uint64_t n;
  DK_HD void put(uint8_t b) { hs.put(b); n++; }
};
struct WriteSink {
  uint8_t* o; int64_t n, cap;
  DK_HD void put(uint8_t b) { if (n < cap) o[n] = b; n++; }
};
struct CmpSink {  // compares the emitted stream with a stored canonical key
  const uint8_t* k; int64_t kn, n; int eq;
  DK_HD void put(uint8_t b) { if (n >= kn || k[n] != b) eq = 0; n++; }
};

// ---- UTF-8 helpers ----
DK_HD int utf8_len_valid(const uint8_t* s, int64_t i, int64_t n, uint32_t* cp) {
  // Returns sequence length if s[i..] is a valid UTF-8 scalar, else 0.
  uint8_t b = s[i];
  if (b < 0x80) { *cp = b; return 1; }
  int need; uint8_t lo = 0x80, hi = 0xBF; uint32_t v;
  if (b >= 0xC2 && b <= 0xDF) { need = 1; v = b & 0x1F; }
  else if (b >= 0xE0 && b <= 0xEF) { need = 2; v = b & 0x0F; if (b == 0xE0) lo = 0xA0; if (b == 0xED) hi = 0x9F; }
  else if (b >= 0xF0 && b <= 0xF4) { need = 3; v = b & 0x07; if (b == 0xF0) lo = 0x90; if (b == 0xF4) hi = 0x8F; }
  else return 0;
  if (i + need >= n + 0 && i + need > n - 1 + 1) return 0;
  for (int k = 1; k <= need; k++) {
    if (i + k >= n) return 0;
    uint8_t c = s[i + k];
    uint8_t l = (k == 1) ? lo : 0x80, h = (k == 1) ? hi : 0xBF;
    if (c < l || c > h) return 0;
    v = (v << 6) | (c & 0x3F);
  }
  *cp = v;
  return need + 1;
}
DK_HD bool java_space(uint32_t c) {
  return c == 0x20 || c == 0xA0 || c == 0x1680 || (c >= 0x2000 && c <= 0x200A) || c == 0x2028 ||
         c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
DK_HD bool java_other_ok(uint32_t c) { return c > 128 && !java_space(c) && !(c <= 0x9F); }

// ---- URI parse (JDK java.net.URI.Parser grammar) ----
struct UriParts {
  int32_t sch_e;           // scheme = [0, sch_e) ; -1 none
  int32_t opaque;
  int32_t ssp_b, ssp_e;
  int32_t auth;            // 0 none, 1 server, 2 registry
  int32_t auth_b, auth_e;
  int32_t ui_b, ui_e;      // -1 none
  int32_t host_b, host_e;
  int64_t port;            // -1 none
  int32_t path_b, path_e;
  int32_t q_b, q_e;        // -1 none
  int32_t f_b, f_e;        // -1 none
};

enum CompClass { K_PATH, K_URIC, K_USERINFO, K_REGNAME, K_SERVER, K_SCOPE };

DK_HD bool comp_ok(uint16_t k, uint8_t c, int cls) {
  switch (cls) {
    case K_PATH: return cc_unres(k) || (k & CC_PATHX);
    case K_URIC: return cc_unres(k) || (k & CC_RESERVED);
    case K_USERINFO: return cc_unres(k) || (k & CC_USERX);
    case K_REGNAME: return cc_unres(k) || (k & CC_REGX);
    case K_SERVER: return cc_unres(k) || (k & (CC_USERX | CC_SERVX)) || c == '-';
    default: return (k & (CC_DIGIT | CC_ALPHA)) || c == '_' || c == '.';
  }
}

struct UriScanner {
  const uint8_t* s; int32_t n; int err;

  // scan [p,e) while chars are allowed (escapes + "other" non-ASCII allowed when esc); -1 on a
  // malformed escape (URISyntaxException "Malformed escape pair")
  DK_HD int32_t scan(int32_t p, int32_t e, int cls, bool esc) {
    while (p < e) {
      uint8_t c = s[p];
      if (c && c < 0x80 && comp_ok(uri_class(c), c, cls)) { p++; continue; }
      if (esc) {
        if (c == '%') {
          if (p + 3 <= e && (uri_class(s[p + 1]) & CC_HEX) && (uri_class(s[p + 2]) & CC_HEX)) { p += 3; continue; }
          return -1;
        }
        if (c >= 0x80) { uint32_t cp; int l = utf8_len_valid(s, p, n, &cp); if (l && java_other_ok(cp)) { p += l; continue; } }
      }
      break;
    }
    return p;
  }
  DK_HD bool check(int32_t p, int32_t e, int cls, bool esc) { return scan(p, e, cls, esc) == e; }
  // first index in [p,e) of a char in `stop`, -1 if a char in `errs` comes first, e if none
  DK_HD int32_t find(int32_t p, int32_t e, const char* errs, const char* stop) {
    for (; p < e; p++) {
      uint8_t c = s[p];
      for (const char* q = errs; *q; q++) if (c == (uint8_t)*q) return -1;
      for (const char* q = stop; *q; q++) if (c == (uint8_t)*q) return p;
    }
    return e;
  }
  DK_HD bool digit(int32_t i) { return (uri_class(s[i]) & CC_DIGIT) != 0; }
  DK_HD bool alnum(int32_t i) { return (uri_class(s[i]) & (CC_DIGIT | CC_ALPHA)) != 0; }

  DK_HD int32_t ipv4(int32_t start, int32_t e) {   // parseIPv4Address: end or -1
    int32_t m = start;
    while (m < e && (digit(m) || s[m] == '.')) m++;
    if (m <= start) return -1;
    int32_t p = start;
    for (int k = 0; k < 4; k++) {
      int32_t q = p; int64_t v = 0;
      while (q < m && digit(q)) { v = v * 10 + (s[q] - '0'); if (v > 255) return -1; q++; }
      if (q <= p) return -1;
      p = q;
      if (k < 3) { if (p < m && s[p] == '.') p++; else return -1; }
    }
    if (p < m) return -1;
    if (p < e && s[p] != ':') return -1;
    return p;
  }
  DK_HD int32_t hostname(int32_t start, int32_t e) {  // parseHostname: end or -1 (error)
    int32_t p = start, l = -1;
    do {
      int32_t q = p;
      while (q < e && alnum(q)) q++;
      if (q <= p) break;
      l = p; p = q;
      q = p;
      while (q < e && (alnum(q) || s[q] == '-')) q++;
      if (q > p) { if (s[q - 1] == '-') return -1; p = q; }
      if (p < e && s[p] == '.') p++; else break;
    } while (p < e);
    if (p < e && s[p] != ':') return -1;
    if (l < 0) return -1;
    if (l > start && !(uri_class(s[l]) & CC_ALPHA)) return -1;
    return p;
  }
  DK_HD bool ipv6(int32_t p, int32_t e) {
    int groups = 0; bool dbl = false; int32_t i = p;
    if (i >= e) return false;
    if (s[i] == ':') { if (i + 1 < e && s[i + 1] == ':') { dbl = true; i += 2; } else return false; }
    while (i < e) {
      int32_t j = i;
      while (j < e && (uri_class(s[j]) & CC_HEX)) j++;
      if (j < e && s[j] == '.') { if (ipv4(i, e) != e) return false; groups += 2; i = e; break; }
      if (j == i || j - i > 4) return false;
      groups++; i = j;
      if (i == e) break;
      if (s[i] != ':') return false;
      i++;
      if (i < e && s[i] == ':') { if (dbl) return false; dbl = true; i++; if (i == e) break; }
      else if (i == e) return false;
    }
    return dbl ? groups <= 7 : groups == 8;
  }
  DK_HD bool server(int32_t p, int32_t e, UriParts& r) {
    int32_t q = find(p, e, "/?#", "@");
    if (q >= p && q < e && s[q] == '@') {
      int32_t x = scan(p, q, K_USERINFO, true);
      if (x != q) return false;
      r.ui_b = p; r.ui_e = q; p = q + 1;
    }
    if (p < e && s[p] == '[') {
      p++;
      q = find(p, e, "/?#", "]");
      if (!(q > p && q < e && s[q] == ']')) return false;
      int32_t rr = find(p, q, "", "%");
      if (rr > p && rr < q) {
        if (!ipv6(p, rr) || rr + 1 == q || !check(rr + 1, q, K_SCOPE, false)) return false;
      } else if (!ipv6(p, q)) return false;
      r.host_b = p - 1; r.host_e = q + 1; p = q + 1;
    } else {
      q = ipv4(p, e);
      if (q <= p) { q = hostname(p, e); if (q < 0) return false; }
      r.host_b = p; r.host_e = q; p = q;
    }
    if (p < e && s[p] == ':') {
      p++;
      q = e;
      if (q > p) {
        int64_t v = 0;
        for (int32_t i = p; i < q; i++) { if (!digit(i)) return false; v = v * 10 + (s[i] - '0'); if (v > 2147483647LL) return false; }
        r.port = v; p = q;
      }
    }
    return p >= e;
  }
  // returns false on URISyntaxException
  DK_HD bool authority(int32_t p, int32_t e, UriParts& r) {
    bool serv = true;
    if (find(p, e, "", "]") > p) {      // JDK: taken unless the authority starts with ']'
      for (int32_t i = p; i < e;) {
        uint8_t c = s[i];
        if (c && c < 0x80 && (comp_ok(uri_class(c), c, K_SERVER) || c == '%')) { i++; continue; }
        if (c >= 0x80) { uint32_t cp; int l = utf8_len_valid(s, i, n, &cp); if (l && java_other_ok(cp)) { i += l; continue; } }
        serv = false; break;
      }
    } else {
      int32_t x = scan(p, e, K_SERVER, true);
      if (x < 0) return false;
      serv = (x == e);
    }
    int32_t x = scan(p, e, K_REGNAME, true);
    if (x < 0) return false;
    bool reg = (x == e);
    r.auth_b = p; r.auth_e = e;
    if (reg && !serv) { r.auth = 2; return true; }
    if (serv) {
      UriParts t = r;
      if (server(p, e, t)) { r = t; r.auth = 1; return true; }
    }
    if (reg) { r.auth = 2; r.ui_b = r.host_b = -1; r.port = -1; return true; }
    return false;
  }
  DK_HD bool hier(int32_t p, UriParts& r, int32_t* outp) {
    if (p + 1 < n && s[p] == '/' && s[p + 1] == '/') {
      p += 2;
      int32_t q = find(p, n, "", "/?#");
      if (q > p) { if (!authority(p, q, r)) return false; p = q; }
      else if (q >= n) return false;
    }
    int32_t q = find(p, n, "", "?#");
    if (!check(p, q, K_PATH, true)) return false;
    r.path_b = p; r.path_e = q; p = q;
    if (p < n && s[p] == '?') {
      p++;
      q = find(p, n, "", "#");
      if (!check(p, q, K_URIC, true)) return false;
      r.q_b = p; r.q_e = q; p = q;
    }
    *outp = p;
    return true;
  }
  DK_HD bool parse(UriParts& r) {
    r.sch_e = -1; r.opaque = 0; r.ssp_b = r.ssp_e = 0; r.auth = 0; r.auth_b = r.auth_e = 0;
    r.ui_b = r.ui_e = -1; r.host_b = r.host_e = -1; r.port = -1; r.path_b = r.path_e = 0;
    r.q_b = r.q_e = -1; r.f_b = r.f_e = -1;
    int32_t p = find(0, n, "/?#", ":");
    if (p >= 0 && p < n && s[p] == ':') {
      if (p == 0 || !(uri_class(s[0]) & CC_ALPHA)) return false;
      for (int32_t i = 1; i < p; i++) {
        uint8_t c = s[i]; uint16_t k = uri_class(c);
        if (!(c < 0x80 && ((k & (CC_DIGIT | CC_ALPHA)) || c == '+' || c == '-' || c == '.'))) return false;
      }
      r.sch_e = p;
      p++;
      if (p < n && s[p] == '/') {
        if (!hier(p, r, &p)) return false;
      } else {
        int32_t q = find(p, n, "", "#");
        if (q <= p) return false;
        if (!check(p, q, K_URIC, true)) return false;
        r.opaque = 1; r.ssp_b = p; r.ssp_e = q; p = q;
      }
    } else {
      if (!hier(0, r, &p)) return false;
    }
    if (p < n && s[p] == '#') {
      if (!check(p + 1, n, K_URIC, true)) return false;
      r.f_b = p + 1; r.f_e = n; p = n;
    }
    return p >= n;
  }
};

template <class Sink>
DK_HD void emit_lower(Sink& k, const uint8_t* s, int32_t b, int32_t e) {
  for (int32_t i = b; i < e; i++) { uint8_t c = s[i]; k.put((c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c); }
}
template <class Sink>
DK_HD void emit_pct(Sink& k, const uint8_t* s, int32_t b, int32_t e) {
  for (int32_t i = b; i < e; i++) {
    uint8_t c = s[i];
    k.put(c);
    if (c == '%' && i + 2 < e) {
      for (int j = 1; j <= 2; j++) { uint8_t d = s[i + j]; k.put((d >= 'A' && d <= 'Z') ? (uint8_t)(d + 32) : d); }
      i += 2;
    }
  }
}

// Is the string a plain relative path (fast path)? Requires valid ASCII only.
DK_HD bool uri_simple(const uint8_t* s, int32_t n) {
  if (n >= 2 && s[0] == '/' && s[1] == '/') return false;
  for (int32_t i = 0; i < n; i++) if (s[i] >= 0x80 || !(uri_class(s[i]) & CC_SIMPLE)) return false;
  return true;
}

// Emit the canonical stream. Returns 0 ok, -1 URISyntaxException, -2 malformed UTF-8 (needs the
// Java replacement pre-pass, see dk_key_repair in the host).
template <class Sink>
DK_HD int uri_emit(const uint8_t* s, int32_t n, Sink& k) {
  if (uri_simple(s, n)) {
    k.put(TAG_PATH);
    for (int32_t i = 0; i < n; i++) k.put(s[i]);
    return 0;
  }
  for (int32_t i = 0; i < n;) {           // malformed UTF-8 is handled by the caller
    if (s[i] < 0x80) { i++; continue; }
    uint32_t cp; int l = utf8_len_valid(s, i, n, &cp);
    if (!l) return -2;
    i += l;
  }
  UriScanner sc{s, n, 0};
  UriParts r;
  if (!sc.parse(r)) return -1;
  if (r.sch_e >= 0) { k.put(TAG_SCHEME); emit_lower(k, s, 0, r.sch_e); }
  if (r.opaque) {
    k.put(TAG_OPAQUE); emit_pct(k, s, r.ssp_b, r.ssp_e);
  } else {
    if (r.auth == 1) {
      k.put(TAG_SERVER);
      if (r.ui_b >= 0) { k.put(TAG_USERINFO); emit_pct(k, s, r.ui_b, r.ui_e); }
      k.put(TAG_HOST); emit_lower(k, s, r.host_b, r.host_e);
      if (r.port >= 0) {
        k.put(TAG_PORT);
        char d[12]; int nd = 0; int64_t v = r.port;
        do { d[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
        while (nd) k.put((uint8_t)d[--nd]);
      }
    } else if (r.auth == 2) {
      k.put(TAG_REGISTRY); emit_pct(k, s, r.auth_b, r.auth_e);
    }
    k.put(TAG_PATH); emit_pct(k, s, r.path_b, r.path_e);
    if (r.q_b >= 0) { k.put(TAG_QUERY); emit_pct(k, s, r.q_b, r.q_e); }
  }
  if (r.f_b >= 0) { k.put(TAG_FRAGMENT); emit_pct(k, s, r.f_b, r.f_e); }
  return 0;
}

// DV unique id stream: 0x01 + storageType + pathOrInlineDv + ("@Optional[" offset "]")
// (or the single byte 0x00 when the action has no deletion vector).
template <class Sink>
DK_HD int dv_emit(bool has_dv, const uint8_t* st, int32_t stn, const uint8_t* pid, int32_t pidn,
                  bool has_off, int32_t off, Sink& k) {
  if (!has_dv) { k.put(0); return 0; }
  for (int32_t i = 0; i < stn;) { if (st[i] < 0x80) { i++; continue; } uint32_t cp; int l = utf8_len_valid(st, i, stn, &cp); if (!l) return -2; i += l; }
  for (int32_t i = 0; i < pidn;) { if (pid[i] < 0x80) { i++; continue; } uint32_t cp; int l = utf8_len_valid(pid, i, pidn, &cp); if (!l) return -2; i += l; }
  k.put(1);
  for (int32_t i = 0; i < stn; i++) k.put(st[i]);
  for (int32_t i = 0; i < pidn; i++) k.put(pid[i]);
  if (has_off) {
    const char* pre = "@Optional[";
    for (const char* q = pre; *q; q++) k.put((uint8_t)*q);
    char d[12]; int nd = 0; int64_t v = off; bool neg = v < 0; if (neg) v = -v;
    do { d[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    if (neg) k.put('-');
    while (nd) k.put((uint8_t)d[--nd]);
    k.put(']');
  }
  return 0;
}

// The dvUniqueId hash of dv_emit + HashSink (DeletionVectorDescriptor.java:167-174), with
// pathOrInlineDv absorbed 8 bytes at a time (aligned loads + funnel shift, appended to the partial
// word: the stream's words are the same, so is the hash). False when storageType or pathOrInlineDv
// holds a non-ASCII byte: dv_emit validates those (the caller falls back to it). The loads may read
// up to 15 bytes past the string: decoded string columns carry 16 bytes of slack (alloc_outputs).
// Host and device (tests/test_dv_hash.py checks it against dv_emit on the host).
DK_HD bool dv_hash_words(const uint8_t* st, int32_t stn, const uint8_t* pid, int32_t pidn,
                                              bool has_off, int32_t off, uint32_t seed, uint64_t* out) {
  Hash64 hs; hs.init(kHashSeed(seed));
  hs.put(1);
  for (int32_t i = 0; i < stn; i++) { if (st[i] >= 0x80) return false; hs.put(st[i]); }
  const uintptr_t pa = (uintptr_t)pid;
  const uint64_t* base = (const uint64_t*)(pa & ~(uintptr_t)7);
  const int sh = (int)(pa & 7) * 8;
  const int32_t nw = (pidn + 7) >> 3;
  uint64_t any = 0;
  for (int32_t j = 0; j < nw; j++) {
    uint64_t w = sh ? (base[j] >> sh) | (base[j + 1] << (64 - sh)) : base[j];
    int nbytes = 8;
    if (j == nw - 1 && (pidn & 7)) { nbytes = pidn & 7; w &= (1ull << (8 * nbytes)) - 1; }
    any |= w;
    const int nb = hs.nb;
    if (nb + nbytes >= 8) {
      hs.word(hs.buf | (w << (8 * nb)));
      hs.buf = nb ? (w >> (64 - 8 * nb)) : 0ull;
      hs.nb = nb + nbytes - 8;
    } else {
      hs.buf |= w << (8 * nb);
      hs.nb = nb + nbytes;
    }
  }
  if (any & 0x8080808080808080ull) return false;
  uint64_t n = 1 + (uint64_t)stn + (uint64_t)pidn;
  if (has_off) {
    const char* pre = "@Optional[";
    for (const char* q = pre; *q; q++) hs.put((uint8_t)*q);
    char d[12]; int nd = 0; int64_t v = off; const bool neg = v < 0; if (neg) v = -v;
    do { d[nd++] = (char)('0' + v % 10); v /= 10; } while (v);
    n += 10 + nd + (neg ? 1 : 0) + 1;
    if (neg) hs.put('-');
    while (nd) hs.put((uint8_t)d[--nd]);
    hs.put(']');
  }
  *out = hs.final_(n);
  return true;
}

// Fast-path character class CC_SIMPLE (unreserved = alnum + "-_.!~*'()", plus "@&=+$,;/"),
// tested 4 bytes at a time: ok(c) = LO[c & 15] & HI[c >> 4] != 0 for c < 0x80, one bit per high
// nibble 2..7 (tables built from the class; the engine re-checks them against uri_class() at
// creation). On the device each 16-entry lookup is two v_perm_b32 + one bit-select for 4 bytes.
DK_HD uint32_t perm8(uint32_t t1, uint32_t t0, uint32_t sel) {   // bytes of sel in 0..7 -> (t1:t0)
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(t1, t0, sel);
#else
  uint64_t t = ((uint64_t)t1 << 32) | t0;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) r |= (uint32_t)((t >> (8 * ((sel >> (8 * i)) & 7))) & 0xff) << (8 * i);
  return r;
#endif
}
DK_HD bool simple4(uint32_t x) {
  if (x & 0x80808080u) return false;
  const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x07070707u;
  const uint32_t l7 = lo & 0x07070707u, m = ((lo >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t rl = (perm8(0x3f3f3e3fu, 0x3e3e3f2eu, l7) & ~m) | (perm8(0x1d351715u, 0x173d3f3fu, l7) & m);
  const uint32_t v = rl & perm8(0x20100804u, 0x02010000u, hi);
  return ((v - 0x01010101u) & ~v & 0x80808080u) == 0;      // every byte non-zero
}
DK_HD bool simple8(uint64_t w) { return simple4((uint32_t)w) && simple4((uint32_t)(w >> 32)); }

// Fast path of path_hash for plain relative paths: the stream is TAG_PATH followed by the raw
// bytes; `load8(j)` returns the little-endian bytes s[8j..8j+8) (bytes past n are ignored).
// Returns false (nothing computed) when the string is not simple (the generic parser decides).
template <class Load8>
DK_HD bool simple_path_hash(int32_t n, const Load8& load8, uint32_t seed, uint64_t* out) {
  Hash64 hs; hs.init(kHashSeed(seed));
  hs.h = Hash64::mixw(hs.h, 0x100u | TAG_PATH);
  const int32_t nfull = n >> 3;
  for (int32_t j = 0; j < nfull; j++) {
    const uint64_t c = load8(j);
    if (!simple8(c) || (j == 0 && (c & 0xffff) == 0x2f2f)) return false;   // leading "//" = authority
    hs.word(c);
  }
  uint64_t tail = 0;
  if (n & 7) {
    const uint64_t mask = (1ull << (8 * (n & 7))) - 1;
    tail = load8(nfull) & mask;
    if (!simple8(tail | (0x6161616161616161ull & ~mask))) return false;     // pad with 'a'
    if (nfull == 0 && n >= 2 && (tail & 0xffff) == 0x2f2f) return false;
  }
  *out = Hash64::fin(hs.h, tail, (uint64_t)n + 1);
  return true;
}

// Hash of a path's canonical stream (generic, byte at a time).
DK_HD int path_hash(const uint8_t* s, int32_t n, uint32_t seed, uint64_t* out) {
  HashSink k; k.hs.init(kHashSeed(seed)); k.n = 0;
  int rc = uri_emit(s, n, k);
  if (rc) return rc;
  *out = k.hs.final_(k.n);
  return 0;
}

}  // namespace dk
