// Predicate compiler behind the C ABI (include/dkgpu.h: dk_skip_compile, dk_part_compile): the two
// predicates a scan hands to ExpressionHandler.getPredicateEvaluator, compiled into the postfix
// programs k_stats_eval / k_stats_parsed / k_parsed_eval and k_part_eval run on the device.
//
//  * data skipping (ScanImpl.applyDataSkipping, KA/internal/ScanImpl.java:304-352): the
//    DataSkippingPredicate DataSkippingUtils.constructDataSkippingFilter built
//    (KA/internal/skipping/DataSkippingUtils.java:156-456), over the pruned stats schema, optionally
//    wrapped as ScanImpl wraps it: =(COALESCE(skip, true), ALWAYS_TRUE);
//  * partition pruning (ScanImpl.applyPartitionPruning, ScanImpl.java:245-294): the partition
//    predicate rewritten over the scan-file schema (PartitionUtils.rewritePartitionPredicateOnScanFileSchema,
//    KA/internal/util/PartitionUtils.java:324-358): element_at(add.partitionValues, <physical name>),
//    wrapped in partition_value(..., <type>) unless the column is a string.
//
// Comparators follow DefaultExpressionEvaluator.transformBinaryComparator (KD/internal/expressions/
// DefaultExpressionEvaluator.java:337-354): operands of different types compare only after an
// ImplicitCastExpression up-cast (ImplicitCastExpression.java:30-41,118-125), otherwise the reference
// throws "Unsupported expression" (status 3 here). Float / double comparisons are planned exactly
// (Float.compare / Double.compare of the value the JSON number or partition string rounds to,
// DefaultExpressionUtils.java:146-153): rounding is monotone, so "round(x) <op> literal" holds on an
// interval of exact values bounded by rounding-cell edges, which the device compares digit by digit.
//
// There are no size caps: programs live in device memory, paths and fields are indexed through
// tables, and AND / OR chains deeper than the device stack are re-associated into balanced trees
// (Kleene AND / OR are associative and commutative, and evaluation has no side effects).
//
// Input format (JSON text; the Java side writes it with an expression visitor):
//   expression := {"col": ["a", "b"]}
//              |  {"lit": <value>, "type": "<Kernel type>"}   value null for a null literal; integral
//                 types, date (epoch days) and timestamps (micros) as JSON integers; string as a JSON
//                 string; decimal(p,s) as the BigDecimal text; float / double as "0x<IEEE bits>" (or a
//                 round-tripping number); boolean as true / false; binary as hex digits
//              |  {"op": "<NAME>", "args": [expression...], "type": "<Kernel type>"}   (type: partition_value)
//   schema     := Kernel StructType JSON ({"type": "struct", "fields": [{"name", "type", ...}]})
#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/dkgpu.h"
#include "dk_device.h"
#include "dk_expr.h"

using namespace dk;

namespace {

// ---------------------------------------------------------------------------------------------
// JSON
// ---------------------------------------------------------------------------------------------
struct JV {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  std::string s;                                 // NUM: the token; STR: decoded UTF-8
  std::vector<JV> a;
  std::vector<std::pair<std::string, JV>> o;
  const JV* get(const char* k) const {
    for (const auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JParse {
  const char* p;
  const char* e;
  std::string err;
  int depth = 0;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
  bool bad(const char* m) { if (err.empty()) err = m; return false; }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp >= 0xD800 && cp <= 0xDFFF) { o += '?'; return; }   // a lone surrogate: String.getBytes(UTF_8)
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
  }
  bool hex4(uint32_t* v) {
    if (e - p < 4) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; k++) {
      const char c = p[k];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= c - '0';
      else if (c >= 'a' && c <= 'f') x |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') x |= c - 'A' + 10;
      else return false;
    }
    p += 4;
    *v = x;
    return true;
  }
  bool str(std::string& o) {
    if (p >= e || *p != '"') return bad("expected a string");
    p++;
    while (p < e && *p != '"') {
      if ((unsigned char)*p < 0x20) return bad("control character in a string");
      if (*p != '\\') { o += *p++; continue; }
      if (++p >= e) return bad("bad escape");
      const char c = *p++;
      switch (c) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return bad("bad \\u escape");
          if (cp >= 0xD800 && cp <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo <= 0xDFFF) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            else p = save;
          }
          utf8(o, cp);
          break;
        }
        default: return bad("bad escape");
      }
    }
    if (p >= e) return bad("unterminated string");
    p++;
    return true;
  }
  bool value(JV& v) {
    ws();
    if (p >= e) return bad("unexpected end of JSON");
    if (++depth > 20000) return bad("JSON nested too deeply");
    const char c = *p;
    bool ok = true;
    if (c == '{') {
      v.t = JV::OBJ;
      p++;
      ws();
      if (p < e && *p == '}') { p++; depth--; return true; }
      while (ok) {
        ws();
        std::string k;
        if (!str(k)) return false;
        ws();
        if (p >= e || *p != ':') return bad("expected ':'");
        p++;
        v.o.emplace_back(std::move(k), JV());
        if (!value(v.o.back().second)) return false;
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') { p++; break; }
        return bad("expected ',' or '}'");
      }
    } else if (c == '[') {
      v.t = JV::ARR;
      p++;
      ws();
      if (p < e && *p == ']') { p++; depth--; return true; }
      while (true) {
        v.a.emplace_back();
        if (!value(v.a.back())) return false;
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; break; }
        return bad("expected ',' or ']'");
      }
    } else if (c == '"') {
      v.t = JV::STR;
      if (!str(v.s)) return false;
    } else if (c == 't' && e - p >= 4 && !strncmp(p, "true", 4)) {
      v.t = JV::BOOL; v.b = true; p += 4;
    } else if (c == 'f' && e - p >= 5 && !strncmp(p, "false", 5)) {
      v.t = JV::BOOL; v.b = false; p += 5;
    } else if (c == 'n' && e - p >= 4 && !strncmp(p, "null", 4)) {
      v.t = JV::NUL; p += 4;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      const char* q = p;
      if (*q == '-') q++;
      if (q >= e || !isdigit((unsigned char)*q)) return bad("bad number");
      while (q < e && isdigit((unsigned char)*q)) q++;
      if (q < e && *q == '.') { q++; if (q >= e || !isdigit((unsigned char)*q)) return bad("bad number"); while (q < e && isdigit((unsigned char)*q)) q++; }
      if (q < e && (*q == 'e' || *q == 'E')) {
        q++;
        if (q < e && (*q == '+' || *q == '-')) q++;
        if (q >= e || !isdigit((unsigned char)*q)) return bad("bad number");
        while (q < e && isdigit((unsigned char)*q)) q++;
      }
      v.t = JV::NUM;
      v.s.assign(p, q);
      p = q;
    } else {
      return bad("unexpected character in JSON");
    }
    depth--;
    return true;
  }
};

bool parse_json(const char* text, JV& out, std::string& err) {
  if (!text) { err = "null JSON text"; return false; }
  JParse P{text, text + strlen(text), {}};
  if (!P.value(out)) { err = P.err; return false; }
  P.ws();
  if (P.p != P.e) { err = "trailing content after the JSON value"; return false; }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Types and schemas
// ---------------------------------------------------------------------------------------------
std::string norm_type(std::string t) {
  for (auto& c : t) c = (char)tolower((unsigned char)c);
  std::string o;
  for (char c : t) if (c != ' ') o += c;
  return o;
}
bool is_decimal(const std::string& t) { return t.compare(0, 7, "decimal") == 0; }
bool is_integral(const std::string& t) { return t == "long" || t == "integer" || t == "short" || t == "byte"; }
bool is_float(const std::string& t) { return t == "float" || t == "double"; }

// ImplicitCastExpression.UP_CASTABLE_TYPE_TABLE (ImplicitCastExpression.java:30-41, canCastTo :118-125)
bool up_cast(const std::string& from, const std::string& to) {
  static const char* order[] = {"byte", "short", "integer", "long", "float", "double"};
  int a = -1, b = -1;
  for (int i = 0; i < 6; i++) { if (from == order[i]) a = i; if (to == order[i]) b = i; }
  return a >= 0 && b >= 0 && a < b;
}
bool comparable(const std::string& a, const std::string& b) { return a == b || up_cast(a, b) || up_cast(b, a); }

typedef std::vector<std::string> Path;

// StructType JSON -> primitive leaf path -> type (nested structs flattened; arrays / maps "complex")
bool walk_schema(const JV& st, Path& prefix, std::vector<std::pair<Path, std::string>>& out, std::string& err) {
  const JV* fields = st.get("fields");
  if (!fields || fields->t != JV::ARR) { err = "schema: a struct needs \"fields\""; return false; }
  for (const JV& f : fields->a) {
    const JV* n = f.get("name");
    const JV* t = f.get("type");
    if (!n || n->t != JV::STR || !t) { err = "schema: a field needs \"name\" and \"type\""; return false; }
    prefix.push_back(n->s);
    if (t->t == JV::STR) {
      out.emplace_back(prefix, norm_type(t->s));
    } else if (t->t == JV::OBJ && t->get("type") && t->get("type")->t == JV::STR && t->get("type")->s == "struct") {
      if (!walk_schema(*t, prefix, out, err)) return false;
    } else {
      out.emplace_back(prefix, "complex");
    }
    prefix.pop_back();
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Expressions
// ---------------------------------------------------------------------------------------------
struct Ex {
  enum K { COL, LIT, CALL } k = LIT;
  Path names;                                    // COL
  std::string type;                              // LIT; PARTITION_VALUE's target type
  bool null = false;                             // LIT
  long long iv = 0;                              // integral / date / timestamp / boolean literal
  uint64_t bits = 0;                             // float / double literal (IEEE bits)
  std::string text;                              // string / binary bytes, decimal text
  std::string name;                              // CALL, upper case
  std::vector<Ex> args;
};

bool parse_int64(const std::string& s, long long* v) {
  if (s.empty()) return false;
  errno = 0;
  char* end = nullptr;
  const long long x = strtoll(s.c_str(), &end, 10);
  if (errno || *end) return false;
  *v = x;
  return true;
}

bool decimal_text_ok(const std::string& s) {         // new BigDecimal(text) grammar (ASCII)
  size_t i = 0;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
  int nd = 0;
  bool dot = false;
  for (; i < s.size() && s[i] != 'e' && s[i] != 'E'; i++) {
    if (s[i] == '.') { if (dot) return false; dot = true; continue; }
    if (!isdigit((unsigned char)s[i])) return false;
    nd++;
  }
  if (!nd) return false;
  if (i < s.size()) {
    i++;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) i++;
    if (i >= s.size()) return false;
    for (; i < s.size(); i++) if (!isdigit((unsigned char)s[i])) return false;
  }
  return true;
}

bool to_expr(const JV& j, Ex& x, std::string& err) {
  if (j.t != JV::OBJ) { err = "expression: expected an object"; return false; }
  if (const JV* c = j.get("col")) {
    x.k = Ex::COL;
    if (c->t != JV::ARR || c->a.empty()) { err = "expression: \"col\" needs a non-empty array of names"; return false; }
    for (const JV& n : c->a) {
      if (n.t != JV::STR) { err = "expression: column names are strings"; return false; }
      x.names.push_back(n.s);
    }
    return true;
  }
  if (const JV* l = j.get("lit")) {
    x.k = Ex::LIT;
    const JV* t = j.get("type");
    if (!t || t->t != JV::STR) { err = "expression: a literal needs \"type\""; return false; }
    x.type = norm_type(t->s);
    if (l->t == JV::NUL) { x.null = true; return true; }
    const std::string& ty = x.type;
    if (is_integral(ty) || ty == "date" || ty == "timestamp" || ty == "timestamp_ntz") {
      if ((l->t != JV::NUM && l->t != JV::STR) || !parse_int64(l->s, &x.iv)) { err = "expression: bad " + ty + " literal"; return false; }
      const long long lo = ty == "integer" || ty == "date" ? INT_MIN : ty == "short" ? -32768 : ty == "byte" ? -128 : LLONG_MIN;
      const long long hi = ty == "integer" || ty == "date" ? INT_MAX : ty == "short" ? 32767 : ty == "byte" ? 127 : LLONG_MAX;
      if (x.iv < lo || x.iv > hi) { err = "expression: " + ty + " literal out of range"; return false; }
    } else if (ty == "boolean") {
      if (l->t != JV::BOOL) { err = "expression: bad boolean literal"; return false; }
      x.iv = l->b;
    } else if (ty == "string") {
      if (l->t != JV::STR) { err = "expression: bad string literal"; return false; }
      x.text = l->s;
    } else if (ty == "binary") {
      if (l->t != JV::STR || l->s.size() % 2) { err = "expression: a binary literal is hex digits"; return false; }
      for (size_t i = 0; i < l->s.size(); i += 2) {
        char b[3] = {l->s[i], l->s[i + 1], 0};
        char* end;
        const long v = strtol(b, &end, 16);
        if (*end) { err = "expression: bad binary literal"; return false; }
        x.text += (char)v;
      }
    } else if (is_decimal(ty)) {
      if ((l->t != JV::NUM && l->t != JV::STR) || !decimal_text_ok(l->s)) { err = "expression: bad decimal literal"; return false; }
      x.text = l->s;
    } else if (is_float(ty)) {
      const bool f32 = ty == "float";
      if (l->t == JV::STR && l->s.size() > 2 && l->s[0] == '0' && (l->s[1] == 'x' || l->s[1] == 'X')) {
        char* end;
        x.bits = strtoull(l->s.c_str() + 2, &end, 16);
        if (*end || (f32 && x.bits > 0xffffffffull)) { err = "expression: bad float bits"; return false; }
      } else if (l->t == JV::NUM || l->t == JV::STR) {
        char* end;
        if (f32) { const float f = strtof(l->s.c_str(), &end); uint32_t b; memcpy(&b, &f, 4); x.bits = b; }
        else { const double d = strtod(l->s.c_str(), &end); memcpy(&x.bits, &d, 8); }
        if (*end) { err = "expression: bad " + ty + " literal"; return false; }
      } else {
        err = "expression: bad " + ty + " literal";
        return false;
      }
    } else {
      err = "expression: literal type " + ty + " is not supported";
      return false;
    }
    return true;
  }
  const JV* op = j.get("op");
  if (!op || op->t != JV::STR) { err = "expression: expected \"col\", \"lit\" or \"op\""; return false; }
  x.k = Ex::CALL;
  for (char c : op->s) x.name += (char)toupper((unsigned char)c);
  if (const JV* t = j.get("type")) { if (t->t == JV::STR) x.type = norm_type(t->s); }
  if (const JV* a = j.get("args")) {
    if (a->t != JV::ARR) { err = "expression: \"args\" must be an array"; return false; }
    for (const JV& c : a->a) {
      x.args.emplace_back();
      if (!to_expr(c, x.args.back(), err)) return false;
    }
  }
  return true;
}

bool is_cmp(const std::string& n) { return n == "<" || n == "<=" || n == ">" || n == ">=" || n == "=" || n == "IS NOT DISTINCT FROM"; }
std::string reverse_cmp(const std::string& n) {
  return n == "<" ? ">" : n == "<=" ? ">=" : n == ">" ? "<" : n == ">=" ? "<=" : n;
}

// ---------------------------------------------------------------------------------------------
// Exact float / double planning (binary formats, dyadic rationals)
// ---------------------------------------------------------------------------------------------
typedef unsigned __int128 u128;
struct Dy {                                          // sign * m * 2^e (m odd, or the zero value)
  int sign = 0;
  u128 m = 0;
  int e = 0;
};
int bitlen(u128 m) { int n = 0; while (m) { m >>= 1; n++; } return n; }
Dy dy_norm(Dy x) {
  if (!x.m) return Dy{};
  while (!(x.m & 1)) { x.m >>= 1; x.e++; }
  if (!x.sign) x.sign = 1;
  return x;
}
Dy dy(int sign, u128 m, int e) { Dy x; x.sign = m ? sign : 0; x.m = m; x.e = e; return dy_norm(x); }
Dy dy_neg(Dy x) { x.sign = -x.sign; return x; }
int dy_cmp_mag(const Dy& a, const Dy& b) {
  if (!a.m || !b.m) return a.m ? 1 : b.m ? -1 : 0;
  const int ta = bitlen(a.m) - 1 + a.e, tb = bitlen(b.m) - 1 + b.e;
  if (ta != tb) return ta < tb ? -1 : 1;
  u128 am = a.m, bm = b.m;
  if (a.e > b.e) am <<= (a.e - b.e); else bm <<= (b.e - a.e);
  return am < bm ? -1 : am > bm ? 1 : 0;
}
int dy_cmp(const Dy& a, const Dy& b) {
  if (a.sign != b.sign) return a.sign < b.sign ? -1 : 1;
  if (!a.sign) return 0;
  const int c = dy_cmp_mag(a, b);
  return a.sign > 0 ? c : -c;
}
Dy dy_mid(const Dy& a, const Dy& b) {                // (a + b) / 2 for non-negative a, b of similar size
  if (!a.m) { Dy x = b; x.e -= 1; return x; }
  if (!b.m) { Dy x = a; x.e -= 1; return x; }
  const int e = a.e < b.e ? a.e : b.e;
  const u128 s = (a.m << (a.e - e)) + (b.m << (b.e - e));
  return dy(1, s, e - 1);
}

struct Fmt { int p, emin_ulp, emax; };
const Fmt F32{24, -149, 127}, F64{53, -1074, 1023};
const Fmt& fmt_of(const std::string& t) { return t == "float" ? F32 : F64; }

Dy max_finite(const Fmt& f) { return dy(1, ((u128)1 << f.p) - 1, f.emax - f.p + 1); }
Dy overflow_threshold(const Fmt& f) { return dy(1, ((u128)1 << (f.p + 1)) - 1, f.emax - f.p); }
int ulp_exp(const Dy& a, const Fmt& f) {
  const int e = bitlen(a.m) - 1 + a.e;
  const int u = e - (f.p - 1);
  return u > f.emin_ulp ? u : f.emin_ulp;
}
// floor(|a| / 2^ue) (small results only)
u128 floor_div_pow2(const Dy& a, int ue) {
  const int sh = a.e - ue;
  if (sh >= 0) return a.m << sh;
  if (-sh >= 128) return 0;
  return a.m >> (-sh);
}
Dy value_of(uint64_t bits, const Fmt& f) {
  const uint64_t biased = bits >> (f.p - 1), frac = bits & ((1ull << (f.p - 1)) - 1);
  if (!biased) return dy(1, frac, f.emin_ulp);
  return dy(1, ((u128)1 << (f.p - 1)) | frac, f.emin_ulp + (int)biased - 1);
}
uint64_t index_of(const Dy& v, const Fmt& f) {     // bit pattern of a non-negative value of the format
  if (!v.m) return 0;
  const int ue = ulp_exp(v, f);
  const u128 m = floor_div_pow2(v, ue);
  if (ue == f.emin_ulp && m < ((u128)1 << (f.p - 1))) return (uint64_t)m;
  const uint64_t biased = (uint64_t)(ue - f.emin_ulp + 1);
  return (biased << (f.p - 1)) | (uint64_t)(m - ((u128)1 << (f.p - 1)));
}
long long max_index(const Fmt& f) { return (long long)index_of(max_finite(f), f); }
uint64_t index_floor(const Dy& a, const Fmt& f) {   // largest non-negative finite value <= a (a >= 0)
  if (a.sign <= 0) return 0;
  if (dy_cmp(a, max_finite(f)) >= 0) return index_of(max_finite(f), f);
  int ue = ulp_exp(a, f);
  u128 m = floor_div_pow2(a, ue);
  if (m >= ((u128)1 << f.p)) { ue++; m = floor_div_pow2(a, ue); }
  return index_of(dy(1, m, ue), f);
}

enum { FV_FIN = 0, FV_NAN, FV_PINF, FV_NINF };
struct FVal { int k = FV_FIN; Dy x; bool negz = false; };

FVal round_exact(const Dy& x, const Fmt& f) {       // round to nearest even
  FVal r;
  if (!x.m) return r;
  Dy a = x;
  a.sign = 1;
  if (dy_cmp(a, overflow_threshold(f)) >= 0) { r.k = x.sign > 0 ? FV_PINF : FV_NINF; return r; }
  const int ue = ulp_exp(a, f);
  const int sh = a.e - ue;
  u128 m;
  if (sh >= 0) {
    m = a.m << sh;
  } else {
    const int s = -sh;
    m = s >= 128 ? 0 : a.m >> s;
    int c;                                             // remainder vs one half
    if (s > 128) c = -1;
    else if (s == 128) c = a.m > ((u128)1 << 127) ? 1 : a.m == ((u128)1 << 127) ? 0 : -1;
    else {
      const u128 rem = a.m & (((u128)1 << s) - 1), half = (u128)1 << (s - 1);
      c = rem > half ? 1 : rem == half ? 0 : -1;
    }
    if (c > 0 || (c == 0 && (m & 1))) m++;
  }
  r.x = dy(x.sign, m, ue);
  r.negz = x.sign < 0 && !m;
  return r;
}

// a literal as a value of the comparison format (widening an integral literal rounds it)
bool literal_value(const Ex& lit, const std::string& target, FVal* out) {
  const std::string& lt = lit.type;
  if (is_float(lt)) {
    const bool f32 = lt == "float";
    const Fmt& f = f32 ? F32 : F64;
    if (target == "float" && lt == "double") return false;
    const uint64_t b = lit.bits;
    const uint64_t sign = f32 ? (b >> 31) & 1 : (b >> 63) & 1;
    const uint64_t mag = f32 ? b & 0x7fffffffull : b & 0x7fffffffffffffffull;
    const uint64_t inf = f32 ? 0x7f800000ull : 0x7ff0000000000000ull;
    FVal v;
    if (mag > inf) v.k = FV_NAN;
    else if (mag == inf) v.k = sign ? FV_NINF : FV_PINF;
    else { v.x = value_of(mag, f); if (sign) v.x = dy_neg(v.x); v.negz = sign && !mag; }
    *out = v;
    return true;
  }
  const long long i = lit.iv;
  const Dy x = dy(i < 0 ? -1 : 1, i < 0 ? (u128)(0ull - (unsigned long long)i) : (u128)i, 0);
  *out = round_exact(x, fmt_of(target));
  return true;
}

int java_compare(const FVal& a, const FVal& b) {     // Float.compare / Double.compare
  auto key = [](const FVal& v) { return v.k == FV_NAN ? 3 : v.k == FV_PINF ? 2 : v.k == FV_NINF ? 0 : 1; };
  const int ka = key(a), kb = key(b);
  if (ka != kb) return ka < kb ? -1 : 1;
  if (ka != 1) return 0;
  const int c = dy_cmp(a.x, b.x);
  if (c) return c;
  const int za = a.negz ? 0 : 1, zb = b.negz ? 0 : 1;
  return za < zb ? -1 : za > zb ? 1 : 0;
}
bool test_op(const std::string& op, int c) {
  return op == "<" ? c < 0 : op == "<=" ? c <= 0 : op == ">" ? c > 0 : op == ">=" ? c >= 0 : c == 0;
}

// rank r of value_fmt: the IEEE bits of +value for r >= 0 (+Infinity = max_index + 1), -1 - bits below
// (-0.0 = -1, -Infinity = -max_index - 2): the Float.compare / Double.compare order, NaN apart
struct RankRun { long long a, b; bool nan, pinf, ninf; };
bool rank_run(const std::string& op, const Ex& lit, const std::string& value_fmt, const std::string& cmp_fmt, RankRun* out) {
  FVal V;
  if (!literal_value(lit, cmp_fmt, &V)) return false;
  FVal s;
  s.k = FV_NAN; out->nan = test_op(op, java_compare(s, V));
  s.k = FV_PINF; out->pinf = test_op(op, java_compare(s, V));
  s.k = FV_NINF; out->ninf = test_op(op, java_compare(s, V));
  const Fmt& f = fmt_of(value_fmt);
  const long long mx = max_index(f), lo_r = -mx - 2, hi_r = mx + 1;
  long long fl;
  bool exact;
  if (V.k == FV_NAN) { fl = hi_r + 1; exact = false; }
  else if (V.k == FV_PINF) { fl = hi_r; exact = true; }
  else if (V.k == FV_NINF) { fl = lo_r; exact = true; }
  else if (!V.x.m) { fl = V.negz ? -1 : 0; exact = true; }
  else if (V.x.sign > 0) {
    if (dy_cmp(V.x, max_finite(f)) > 0) { fl = mx; exact = false; }
    else { fl = (long long)index_floor(V.x, f); exact = dy_cmp(value_of((uint64_t)fl, f), V.x) == 0; }
  } else {
    const Dy a = dy_neg(V.x);
    if (dy_cmp(a, max_finite(f)) > 0) { fl = lo_r; exact = false; }
    else {
      const long long g = (long long)index_floor(a, f);
      exact = dy_cmp(value_of((uint64_t)g, f), a) == 0;
      fl = exact ? -g - 1 : -g - 2;
    }
  }
  long long a, b;
  if (op == "<") { a = lo_r; b = exact ? fl - 1 : fl; }
  else if (op == "<=") { a = lo_r; b = fl; }
  else if (op == ">") { a = fl + 1; b = hi_r; }
  else if (op == ">=") { a = exact ? fl : fl + 1; b = hi_r; }
  else { if (exact) a = b = fl; else { a = 1; b = 0; } }
  if (a < lo_r) a = lo_r;
  if (b > hi_r) b = hi_r;
  if (a > b) { a = 1; b = 0; }
  out->a = a; out->b = b;
  return true;
}

// rounding cell of rank r: the exact values that round to it
struct Cell { bool lo_unb = false, hi_unb = false, lo_inc = false, hi_inc = false; Dy lo, hi; };
Cell cell(long long r, const Fmt& f) {
  const long long mx = max_index(f);
  const Dy T = overflow_threshold(f);
  Cell c;
  if (r == mx + 1) { c.lo = T; c.lo_inc = true; c.hi_unb = true; return c; }
  if (r == -mx - 2) { c.lo_unb = true; c.hi = dy_neg(T); c.hi_inc = true; return c; }
  const bool negz = r < 0;
  const uint64_t i = (uint64_t)(r >= 0 ? r : -r - 1);
  if (!i) {
    Dy h = value_of(1, f);
    h.e -= 1;                                        // half the smallest subnormal; ties go to zero
    if (!negz) { c.lo = Dy{}; c.lo_inc = true; c.hi = h; c.hi_inc = true; }
    else { c.lo = dy_neg(h); c.lo_inc = true; c.hi = Dy{}; c.hi_inc = false; }
    return c;
  }
  const Dy mag = value_of(i, f);
  const bool even = !(i & 1);
  const Dy lo = dy_mid(value_of(i - 1, f), mag);
  const Dy hi = (long long)i < mx ? dy_mid(mag, value_of(i + 1, f)) : T;
  const bool hi_inc = even && (long long)i < mx;
  if (!negz) { c.lo = lo; c.lo_inc = even; c.hi = hi; c.hi_inc = hi_inc; }
  else { c.lo = dy_neg(hi); c.lo_inc = hi_inc; c.hi = dy_neg(lo); c.hi_inc = even; }
  return c;
}

enum { C_ALL = 0, C_NONE, C_LT, C_LE, C_GT, C_GE };
struct Cond { int k; Dy B; };
bool plan(const std::string& op, const Ex& lit, const std::string& value_fmt, const std::string& cmp_fmt,
          std::vector<Cond>* conds, RankRun* rr) {
  if (!rank_run(op, lit, value_fmt, cmp_fmt, rr)) return false;
  const Fmt& f = fmt_of(value_fmt);
  const long long mx = max_index(f), lo_r = -mx - 2, hi_r = mx + 1;
  conds->clear();
  if (rr->a > rr->b) { conds->push_back({C_NONE, Dy{}}); return true; }
  if (rr->a > lo_r) { const Cell c = cell(rr->a, f); conds->push_back({c.lo_inc ? C_GE : C_GT, c.lo}); }
  if (rr->b < hi_r) { const Cell c = cell(rr->b, f); conds->push_back({c.hi_inc ? C_LE : C_LT, c.hi}); }
  if (conds->empty()) conds->push_back({C_ALL, Dy{}});
  return true;
}

// exact decimal text of a dyadic rational; scientific notation when shorter (thresholds near the
// subnormal range have hundreds of leading zeros)
std::string decimal_text(const Dy& q) {
  if (!q.m) return "0";
  std::vector<uint32_t> limbs;                       // base 1e9, little-endian
  u128 m = q.m;
  while (m) { limbs.push_back((uint32_t)(m % 1000000000u)); m /= 1000000000u; }
  auto mul = [&](uint64_t k) {
    uint64_t carry = 0;
    for (auto& l : limbs) { const uint64_t t = (uint64_t)l * k + carry; l = (uint32_t)(t % 1000000000u); carry = t / 1000000000u; }
    while (carry) { limbs.push_back((uint32_t)(carry % 1000000000u)); carry /= 1000000000u; }
  };
  int k = 0;                                         // value = digits * 10^-k
  if (q.e >= 0) { for (int e = q.e; e > 0; e -= 29) mul(1ull << (e < 29 ? e : 29)); }
  else {
    k = -q.e;
    int r = k;
    for (; r >= 13; r -= 13) mul(1220703125ull);    // 5^13
    uint64_t p = 1;
    while (r--) p *= 5;
    mul(p);
  }
  std::string s = std::to_string(limbs.back());
  char b[16];
  for (size_t i = limbs.size() - 1; i-- > 0;) { snprintf(b, sizeof b, "%09u", limbs[i]); s += b; }
  const std::string sign = q.sign < 0 ? "-" : "";
  std::string plain = s;
  if (k) {
    if ((int)plain.size() < k + 1) plain = std::string(k + 1 - plain.size(), '0') + plain;
    plain = plain.substr(0, plain.size() - k) + "." + plain.substr(plain.size() - k);
    while (!plain.empty() && plain.back() == '0') plain.pop_back();
    if (!plain.empty() && plain.back() == '.') plain.pop_back();
  }
  std::string sig = s;
  while (sig.size() > 1 && sig.back() == '0') sig.pop_back();
  const long long exp = (long long)s.size() - 1 - k;
  std::string sci = sig.substr(0, 1) + (sig.size() > 1 ? "." + sig.substr(1) : "") + "E" + std::to_string(exp);
  return sign + (sci.size() < plain.size() ? sci : plain);
}

// the conditions over integer x: [lo, hi] inclusive (false: empty)
bool integral_bounds(const std::vector<Cond>& conds, long long* lo, long long* hi) {
  __int128 a = LLONG_MIN, b = LLONG_MAX;
  const __int128 BIG = (__int128)1 << 100;
  auto floor_ = [&](const Dy& B) -> __int128 {
    if (!B.m) return 0;
    if (B.e >= 0) {
      if (bitlen(B.m) + B.e > 100) return B.sign > 0 ? BIG : -BIG;
      const __int128 v = (__int128)(B.m << B.e);
      return B.sign > 0 ? v : -v;
    }
    const int s = -B.e;
    const u128 q = s >= 128 ? 0 : B.m >> s;
    const bool frac = s >= 128 ? true : (B.m & (((u128)1 << s) - 1)) != 0;
    return B.sign > 0 ? (__int128)q : -(__int128)q - (frac ? 1 : 0);
  };
  auto ceil_ = [&](const Dy& B) -> __int128 { return -floor_(dy_neg(B)); };
  for (const Cond& c : conds) {
    if (c.k == C_ALL) continue;
    if (c.k == C_NONE) return false;
    if (c.k == C_LT) { const __int128 v = ceil_(c.B) - 1; if (v < b) b = v; }
    else if (c.k == C_LE) { const __int128 v = floor_(c.B); if (v < b) b = v; }
    else if (c.k == C_GT) { const __int128 v = floor_(c.B) + 1; if (v > a) a = v; }
    else { const __int128 v = ceil_(c.B); if (v > a) a = v; }
  }
  if (a > b) return false;
  *lo = (long long)a;
  *hi = (long long)b;
  return true;
}

// ---------------------------------------------------------------------------------------------
// Program building
// ---------------------------------------------------------------------------------------------
struct Op {
  int32_t op = 0, arg = 0;
  int64_t lit = 0;
  bool has_bytes = false;                            // literal bytes (appended to the pool at finalize)
  std::string bytes;
  bool ranks = false;                                // skipping FCMP: the rank run follows the text
  long long r0 = 1, r1 = 0;
};

const int kMaxStack = 32;                            // SK_STACK / PP_STACK (dk_device.h)

struct Unsupported { int code; std::string msg; };  // 3: the reference throws; 1: not compilable

[[noreturn]] void unsupported_expr(const std::string& n, const std::string& lt, const std::string& rt) {
  throw Unsupported{3, "Unsupported expression: " + n + ": operands are of different types which are not "
                       "comparable: left type=" + lt + ", right type=" + rt};
}
[[noreturn]] void refuse(const std::string& m) { throw Unsupported{1, m}; }

// Re-associate chains of one Kleene connective into a balanced tree (needed only when the natural
// postfix order would overflow the device stack)
void flatten(const Ex& x, const std::string& name, std::vector<const Ex*>& out) {
  if (x.k == Ex::CALL && x.name == name && x.args.size() == 2) { flatten(x.args[0], name, out); flatten(x.args[1], name, out); }
  else out.push_back(&x);
}
Ex balanced(const std::vector<const Ex*>& xs, size_t a, size_t b, const std::string& name, Ex (*rebuild)(const Ex&)) {
  if (b - a == 1) return rebuild(*xs[a]);
  const size_t m = (a + b) / 2;
  Ex n;
  n.k = Ex::CALL;
  n.name = name;
  n.args.push_back(balanced(xs, a, m, name, rebuild));
  n.args.push_back(balanced(xs, m, b, name, rebuild));
  return n;
}
Ex rebalance(const Ex& x) {
  if (x.k == Ex::CALL && (x.name == "AND" || x.name == "OR") && x.args.size() == 2) {
    std::vector<const Ex*> xs;
    flatten(x, x.name, xs);
    return balanced(xs, 0, xs.size(), x.name, rebalance);
  }
  Ex y = x;
  for (auto& c : y.args) c = rebalance(c);
  return y;
}

// stack depth of a postfix sequence (pushes: operands; FCMP / TIMEADD / unary ops keep the depth)
int depth_of(const std::vector<Op>& ops, bool skipping) {
  int d = 0, hi = 0;
  for (const Op& o : ops) {
    int delta;
    if (skipping) {
      delta = (o.op == OP_STAT || o.op == OP_LIT || o.op == OP_LIT_STR || o.op == OP_LIT_DEC) ? 1
            : (o.op == OP_TIMEADD || o.op == OP_FCMP) ? 0 : -1;
    } else {
      delta = (o.op == PO_FIELD || o.op == PO_LIT_INT || o.op == PO_LIT_STR || o.op == PO_LIT_NULL || o.op == PO_LIT_DEC) ? 1
            : (o.op == PO_ISNULL || o.op == PO_ISNOTNULL || o.op == PO_NOT || o.op == PO_FCMP || o.op == PO_STARTS_WITH ||
               o.op == PO_LIKE || o.op == PO_SUBSTR) ? 0
            : o.op == PO_COALESCE ? 1 - o.arg : -1;
    }
    d += delta;
    if (d > hi) hi = d;
  }
  return hi;
}

// --------------------------------------------------------------------------------------------- skipping
struct SkipCompiler {
  std::map<Path, std::string> schema;               // stats leaf -> Kernel type
  std::vector<Path> paths;
  std::vector<Op> ops;

  std::string col_type(const Ex& c) {
    auto it = schema.find(c.names);
    if (it == schema.end()) {
      std::string n;
      for (auto& s : c.names) n += (n.empty() ? "" : ".") + s;
      refuse("data skipping: column " + n + " is not in the stats schema");
    }
    return it->second;
  }
  std::string type_of(const Ex& x) {
    if (x.k == Ex::COL) return col_type(x);
    if (x.k == Ex::LIT) return x.type;
    if (x.name == "TIMEADD") return type_of(x.args.at(0));
    return "boolean";
  }
  void check(const Ex& x) {                          // shape + DefaultExpressionEvaluator type rules
    if (x.k != Ex::CALL) refuse("data skipping: the filter must be a predicate");
    if (x.name == "AND" || x.name == "OR") {
      if (x.args.size() != 2) refuse("data skipping: " + x.name + " takes two predicates");
      for (auto& c : x.args) {
        if (c.k != Ex::CALL || !(c.name == "AND" || c.name == "OR" || is_cmp(c.name)))
          refuse("data skipping: unexpected operand of " + x.name);
        check(c);
      }
      return;
    }
    if (!is_cmp(x.name) || x.name == "IS NOT DISTINCT FROM" || x.args.size() != 2)
      refuse("data skipping: " + x.name + " is not a data-skipping comparison");
    for (auto& c : x.args) {
      if (c.k == Ex::CALL) {
        if (c.name != "TIMEADD" || c.args.size() != 2 || c.args[0].k != Ex::COL || c.args[1].k != Ex::LIT ||
            c.args[1].null || c.args[1].type != "long")
          refuse("data skipping: unexpected operand " + c.name);
        const std::string t = col_type(c.args[0]);
        if (t != "timestamp" && t != "timestamp_ntz") refuse("data skipping: TIMEADD over a " + t + " column");
      } else if (c.k == Ex::COL) {
        const std::string t = col_type(c);
        if (!(is_integral(t) || is_float(t) || is_decimal(t) || t == "date" || t == "string" || t == "timestamp" ||
              t == "timestamp_ntz"))
          refuse("data skipping on " + t + " stats is not supported");
      }
    }
    const std::string lt = type_of(x.args[0]), rt = type_of(x.args[1]);
    if (!comparable(lt, rt)) unsupported_expr(x.name, lt, rt);
  }
  void collect(const Ex& x) {
    if (x.k == Ex::COL) {
      for (auto& p : paths) if (p == x.names) return;
      paths.push_back(x.names);
      return;
    }
    for (auto& c : x.args) collect(c);
  }
  int path_index(const Path& p) {
    for (size_t i = 0; i < paths.size(); i++) if (paths[i] == p) return (int)i;
    refuse("data skipping: internal path error");
  }
  void push(int op, int arg = 0, int64_t lit = 0) { Op o; o.op = op; o.arg = arg; o.lit = lit; ops.push_back(o); }
  void push_bytes(int op, const std::string& b) { Op o; o.op = op; o.has_bytes = true; o.bytes = b; ops.push_back(o); }
  void emit(const Ex& n) {
    if (n.k == Ex::COL) { push(OP_STAT, path_index(n.names)); return; }
    if (n.k == Ex::LIT) {
      if (n.null) { push(OP_LIT, 1, 0); return; }
      if (is_decimal(n.type)) { push_bytes(OP_LIT_DEC, n.text); return; }
      if (n.type == "string") { push_bytes(OP_LIT_STR, n.text); return; }
      if (is_integral(n.type) || n.type == "date" || n.type == "timestamp" || n.type == "timestamp_ntz") { push(OP_LIT, 0, n.iv); return; }
      refuse("data skipping with a " + n.type + " literal is not supported");
    }
    if (n.name == "AND" || n.name == "OR") {
      emit(n.args[0]);
      emit(n.args[1]);
      push(n.name == "AND" ? OP_AND : OP_OR);
      return;
    }
    if (n.name == "TIMEADD") {                       // max + 1 ms (StatsSchemaHelper.java:154-159), in micros
      emit(n.args[0]);
      if (n.args[1].iv > LLONG_MAX / 1000 || n.args[1].iv < LLONG_MIN / 1000) refuse("TIMEADD out of range");
      push(OP_TIMEADD, 0, n.args[1].iv * 1000);
      return;
    }
    if (is_float(type_of(n.args[0])) || is_float(type_of(n.args[1]))) { emit_float(n); return; }
    emit(n.args[0]);
    emit(n.args[1]);
    const std::string& c = n.name;
    push(c == "<" ? OP_LT : c == "<=" ? OP_LE : c == ">" ? OP_GT : c == ">=" ? OP_GE : OP_EQ);
  }
  // a comparison in float / double: integral stats get integer bounds, float / double stats an FCMP
  // per bound (binfloat plan), with the same comparison as a rank run for add.stats_parsed's floats
  void emit_float(const Ex& n) {
    std::string op = n.name;
    const Ex* stat = &n.args[0];
    const Ex* lit = &n.args[1];
    if (stat->k == Ex::LIT && lit->k != Ex::LIT) { std::swap(stat, lit); op = reverse_cmp(op); }
    if (stat->k != Ex::COL || lit->k != Ex::LIT) refuse("data skipping: a float comparison needs a stat and a literal");
    const std::string st = type_of(*stat), lt = lit->type;
    auto cmp_op = [](const std::string& c) { return c == "<" ? OP_LT : c == "<=" ? OP_LE : c == ">" ? OP_GT : c == ">=" ? OP_GE : OP_EQ; };
    if (lit->null) { emit(*stat); push(OP_LIT, 1, 0); push(cmp_op(op)); return; }
    const std::string cmp_t = st == lt ? st : (up_cast(st, lt) ? lt : st);
    const std::string value_fmt = is_float(st) ? st : cmp_t;
    std::vector<Cond> conds;
    RankRun rr;
    if (!plan(op, *lit, value_fmt, cmp_t, &conds, &rr)) refuse("data skipping: float literal narrowed");
    if (!is_float(st)) {
      long long a, b;
      std::vector<std::pair<int, long long>> parts;
      if (!integral_bounds(conds, &a, &b)) parts.push_back({OP_LT, LLONG_MIN});       // never (null when null)
      else {
        if (a > LLONG_MIN) parts.push_back({OP_GE, a});
        if (b < LLONG_MAX) parts.push_back({OP_LE, b});
        if (parts.empty()) parts.push_back({OP_GE, LLONG_MIN});                        // always
      }
      for (size_t k = 0; k < parts.size(); k++) {
        emit(*stat);
        push(OP_LIT, 0, parts[k].second);
        push(parts[k].first);
        if (k) push(OP_AND);
      }
      return;
    }
    const int flags = ((int)rr.nan << 4) | ((int)rr.pinf << 5) | ((int)rr.ninf << 6);
    for (size_t k = 0; k < conds.size(); k++) {
      emit(*stat);
      Op o;
      o.op = OP_FCMP;
      o.has_bytes = true;
      o.ranks = true;
      o.r0 = rr.a; o.r1 = rr.b;
      const Cond& c = conds[k];
      if (c.k == C_ALL || c.k == C_NONE) o.arg = flags | (c.k == C_ALL ? FC_ALL : FC_NONE);
      else {
        o.arg = flags | (c.k == C_LT ? FC_LT : c.k == C_LE ? FC_LE : c.k == C_GT ? FC_GT : FC_GE);
        o.bytes = decimal_text(c.B);
      }
      ops.push_back(o);
      if (k) push(OP_AND);
    }
  }
};

const Ex* unwrap_skipping(const Ex& x) {
  // =(COALESCE(skip, true), ALWAYS_TRUE) (ScanImpl.java:318-324) or COALESCE(skip, true)
  const Ex* p = &x;
  if (p->k == Ex::CALL && p->name == "=" && p->args.size() == 2 && p->args[1].k == Ex::CALL &&
      p->args[1].name == "ALWAYS_TRUE")
    p = &p->args[0];
  if (p->k == Ex::CALL && p->name == "COALESCE" && p->args.size() == 2 && p->args[1].k == Ex::LIT &&
      p->args[1].type == "boolean" && !p->args[1].null && p->args[1].iv == 1)
    p = &p->args[0];
  return p;
}

int sk_type_code(const std::string& t) {
  if (t == "long") return SK_LONG;
  if (t == "integer") return SK_INT;
  if (t == "short") return SK_SHORT;
  if (t == "byte") return SK_BYTE;
  if (t == "date") return SK_DATE;
  if (t == "string") return SK_STRING;
  if (t == "timestamp") return SK_TIMESTAMP;
  if (is_decimal(t)) return SK_DECIMAL;
  if (t == "timestamp_ntz") return SK_TIMESTAMP_NTZ;
  if (t == "float") return SK_FLOAT;
  if (t == "double") return SK_DOUBLE;
  return -1;
}

// --------------------------------------------------------------------------------------------- partitions
struct PartCompiler {
  std::vector<std::pair<std::string, std::string>> used;   // (physical name, normalized type)
  std::vector<std::string> types_full;                     // the Kernel type of each field
  std::vector<Op> ops;
  void push(int op, int arg = 0, int64_t lit = 0) { Op o; o.op = op; o.arg = arg; o.lit = lit; ops.push_back(o); }
  void push_bytes(int op, const std::string& b) { Op o; o.op = op; o.has_bytes = true; o.bytes = b; ops.push_back(o); }

  // element_at(add.partitionValues, 'name') [wrapped in partition_value(.., type)]: (phys, full type)
  bool field_ref(const Ex& x, std::string* phys, std::string* type) {
    const Ex* ea = &x;
    std::string t = "string";
    if (x.k == Ex::CALL && x.name == "PARTITION_VALUE") {
      if (x.args.size() != 1 || x.type.empty()) refuse("partition_value needs one argument and a type");
      ea = &x.args[0];
      t = x.type;
    }
    if (!(ea->k == Ex::CALL && ea->name == "ELEMENT_AT" && ea->args.size() == 2)) return false;
    const Ex& m = ea->args[0];
    const Ex& k = ea->args[1];
    if (!(m.k == Ex::COL && m.names.size() == 2 && m.names[0] == "add" && m.names[1] == "partitionValues") ||
        !(k.k == Ex::LIT && k.type == "string" && !k.null))
      refuse("element_at over anything but add.partitionValues is not a partition filter");
    *phys = k.text;
    *type = t;
    return true;
  }
  int field(const std::string& phys, const std::string& t_full) {
    std::string t = is_decimal(t_full) ? "decimal" : t_full == "timestamp_ntz" ? "timestamp" : t_full == "binary" ? "string" : t_full;
    static const char* known[] = {"long", "integer", "short", "byte", "string", "date", "decimal", "boolean", "float", "double", "timestamp"};
    bool ok = false;
    for (auto k : known) ok = ok || t == k;
    if (!ok) refuse("partition pruning on " + t_full + " column " + phys + " is not supported by this engine build");
    for (size_t i = 0; i < used.size(); i++) if (used[i].first == phys && used[i].second == t) return (int)i;
    used.push_back({phys, t});
    types_full.push_back(t_full);
    return (int)used.size() - 1;
  }
  static std::string kind_of(const std::string& t) {    // comparison kind of a Kernel type
    if (t == "string" || t == "binary") return "string";
    if (t == "date") return "date";
    if (is_decimal(t)) return "decimal";
    if (t == "boolean") return "boolean";
    if (t == "timestamp" || t == "timestamp_ntz") return "timestamp";
    if (is_float(t)) return "float";
    return "integral";
  }
  std::string type_of(const Ex& x) {
    std::string phys, t;
    if (field_ref(x, &phys, &t)) return t;
    if (x.k == Ex::LIT) return x.type;
    if (x.k == Ex::CALL && x.name == "COALESCE" && !x.args.empty()) return type_of(x.args[0]);
    if (x.k == Ex::CALL && x.name == "SUBSTRING") return "string";
    if (x.k == Ex::CALL && x.name == "TIMEADD" && !x.args.empty()) return type_of(x.args[0]);
    return "boolean";
  }
  // stack slots an expression needs as emitted (AND / OR take their deeper operand first: Kleene AND /
  // OR are commutative and both operands are always evaluated, so any nesting -- e.g. a long chain of
  // AND(x, NOT(AND(y, NOT(...)))) -- fits the device stack)
  int need(const Ex& x) {
    if (x.k != Ex::CALL) return 1;
    const std::string& n = x.name;
    const auto& c = x.args;
    if (n == "PARTITION_VALUE" || n == "ELEMENT_AT" || c.empty()) return 1;
    if ((n == "AND" || n == "OR") && c.size() == 2) {
      const int a = need(c[0]), b = need(c[1]);
      return a >= b ? std::max(a, b + 1) : std::max(b, a + 1);
    }
    int d = 0;
    for (size_t i = 0; i < c.size(); i++) d = std::max(d, need(c[i]) + (int)i);
    return std::max(d, 1);
  }
  // an operand (value expression); returns its comparison kind ("" for a null literal)
  std::string operand(const Ex& x) {
    std::string phys, t;
    if (field_ref(x, &phys, &t)) { push(PO_FIELD, field(phys, t)); return kind_of(t); }
    if (x.k == Ex::LIT) {
      if (x.null) { push(PO_LIT_NULL); return ""; }
      const std::string& ty = x.type;
      if (ty == "string" || ty == "binary") { push_bytes(PO_LIT_STR, x.text); return "string"; }
      if (is_decimal(ty)) { push_bytes(PO_LIT_DEC, x.text); return "decimal"; }
      if (ty == "boolean") { push(PO_LIT_INT, 0, x.iv); return "boolean"; }
      if (is_integral(ty) || ty == "date" || ty == "timestamp" || ty == "timestamp_ntz") { push(PO_LIT_INT, 0, x.iv); return kind_of(ty); }
      refuse("partition pruning with a " + ty + " literal is not supported");
    }
    if (x.k == Ex::CALL && x.name == "COALESCE") {   // DefaultExpressionEvaluator.visitCoalesce :236-257
      if (x.args.empty()) throw Unsupported{3, "Unsupported expression: Coalesce requires at least one expression"};
      std::string k0, t0 = type_of(x.args[0]);
      if (t0 != "boolean") throw Unsupported{3, "Unsupported expression: Coalesce is only supported for boolean type expressions"};
      for (auto& a : x.args) {
        if (type_of(a) != t0)
          throw Unsupported{3, "Unsupported expression: Coalesce is only supported for arguments of the same type"};
        const std::string k = is_predicate(a) ? (pred(a), "boolean") : operand(a);
        if (!k.empty()) k0 = k;
      }
      push(PO_COALESCE, (int)x.args.size());
      return k0;
    }
    if (x.k == Ex::CALL && x.name == "TIMEADD") {    // DefaultExpressionEvaluator.visitTimeAdd (:260-288, :593-626)
      if (x.args.size() != 2)
        throw Unsupported{3, "Unsupported expression: TIMEADD requires exactly two arguments: timestamp column and milliseconds"};
      const std::string t0 = type_of(x.args[0]), t1 = type_of(x.args[1]);
      if (!((t0 == "timestamp" || t0 == "timestamp_ntz") && t1 == "long"))
        throw Unsupported{3, "TIMEADD requires a timestamp and a Long (milliseconds) to add to it"};
      operand(x.args[0]);
      operand(x.args[1]);
      push(PO_TIMEADD);
      return "timestamp";
    }
    if (x.k == Ex::CALL && x.name == "SUBSTRING") {  // SubstringEvaluator.java:36-60
      if (x.args.size() < 2 || x.args.size() > 3)
        throw Unsupported{3, "Unsupported expression: Invalid number of inputs to SUBSTRING expression"};
      if (type_of(x.args[0]) != "string")
        throw Unsupported{3, "Unsupported expression: Invalid type of first input of SUBSTRING: expects STRING"};
      for (size_t k = 1; k < x.args.size(); k++) {
        const Ex& a = x.args[k];
        if (!(a.k == Ex::LIT && a.type == "integer" && !a.null))
          throw Unsupported{3, std::string("Unsupported expression: Invalid `") + (k == 1 ? "pos" : "len") +
                               "` argument type for SUBSTRING"};
      }
      operand(x.args[0]);
      const int64_t pos = (uint32_t)(int32_t)x.args[1].iv;
      const int64_t len = x.args.size() == 3 ? x.args[2].iv : 0;
      push(PO_SUBSTR, x.args.size() == 3 ? 1 : 0, pos | (int64_t)((uint64_t)(uint32_t)(int32_t)len << 32));
      return "string";
    }
    if (is_predicate(x)) { pred(x); return "boolean"; }
    refuse("partition pruning on expression " + x.name + " is not supported by this engine build");
  }
  // LIKE pattern -> tokens (LikeExpressionEvaluator.escapeLikeRegex :155-186): '_' one code point,
  // '%' any run, escape + (_ | % | escape) that character, any other escape an error
  static std::string like_tokens(const std::string& pat, uint32_t esc) {
    std::string t;
    std::vector<uint32_t> cps;                       // the pattern's code points (UTF-8 decoded)
    std::vector<std::string> raw;
    for (size_t i = 0; i < pat.size();) {
      const unsigned char c = pat[i];
      const size_t n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
      uint32_t cp = n == 1 ? c : n == 2 ? (c & 31) : n == 3 ? (c & 15) : (c & 7);
      for (size_t k = 1; k < n && i + k < pat.size(); k++) cp = (cp << 6) | (pat[i + k] & 63);
      cps.push_back(cp);
      raw.push_back(pat.substr(i, n));
      i += n;
    }
    for (size_t i = 0; i < cps.size(); i++) {
      if (cps[i] == esc) {
        if (i + 1 == cps.size() || !(cps[i + 1] == '_' || cps[i + 1] == '%' || cps[i + 1] == esc))
          throw Unsupported{3, "LIKE expression has invalid escape sequence: " + pat};
        for (unsigned char b : raw[i + 1]) { t += '\0'; t += (char)b; }
        i++;
      } else if (cps[i] == '_') {
        t += '\1'; t += '\0';
      } else if (cps[i] == '%') {
        t += '\2'; t += '\0';
      } else {
        for (unsigned char b : raw[i]) { t += '\0'; t += (char)b; }
      }
    }
    return t;
  }
  // STARTS_WITH(s, literal) / LIKE(s, pattern[, escape]) (StartsWithExpressionEvaluator.java:38-60,
  // LikeExpressionEvaluator.java:40-80): string inputs, literal second (and third) arguments
  void string_pred(const Ex& x) {
    const bool like = x.name == "LIKE";
    if (like ? (x.args.size() < 2 || x.args.size() > 3) : x.args.size() != 2)
      throw Unsupported{3, "Unsupported expression: Invalid number of inputs to " + x.name + " expression"};
    for (size_t k = 0; k < 2; k++)
      if (type_of(x.args[k]) != "string")
        throw Unsupported{3, like ? "Unsupported expression: LIKE is only supported for string type expressions"
                                  : "Unsupported expression: 'STARTS_WITH' expects STRING type inputs"};
    const Ex& lit = x.args[1];
    if (lit.k != Ex::LIT && !like)
      throw Unsupported{3, "Unsupported expression: 'STARTS_WITH' expects literal as the second input"};
    uint32_t esc = '\\';
    if (x.args.size() == 3) {
      const Ex& e = x.args[2];
      if (!(e.k == Ex::LIT && e.type == "string"))
        throw Unsupported{3, "Unsupported expression: LIKE expects escape token expression to be a literal of String type"};
      const std::string& t = e.text;             // one UTF-16 unit: a BMP code point
      const unsigned char c = t.empty() ? 0 : t[0];
      const size_t n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
      if (e.null || t.empty() || t.size() != n || n == 4)
        throw Unsupported{3, "Unsupported expression: LIKE expects escape token to be a single character"};
      esc = n == 1 ? c : n == 2 ? (c & 31) : (c & 15);
      for (size_t k = 1; k < n; k++) esc = (esc << 6) | (t[k] & 63);
    }
    operand(x.args[0]);
    if (lit.k != Ex::LIT) {                          // a per-row pattern: tokenized on the device per row
      operand(lit);
      push(PO_LIKE_DYN, (int)esc);
      return;
    }
    Op o;
    o.op = like ? PO_LIKE : PO_STARTS_WITH;
    if (lit.null) { o.arg = 1; ops.push_back(o); return; }
    o.has_bytes = true;
    o.bytes = like ? like_tokens(lit.text, esc) : lit.text;
    ops.push_back(o);
  }
  static bool is_predicate(const Ex& x) {
    if (x.k != Ex::CALL) return false;
    const std::string& n = x.name;
    return n == "AND" || n == "OR" || n == "NOT" || n == "IS_NULL" || n == "IS_NOT_NULL" || is_cmp(n) ||
           n == "ALWAYS_TRUE" || n == "ALWAYS_FALSE" || n == "STARTS_WITH" || n == "LIKE";
  }
  void pred(const Ex& x) {
    if (x.k == Ex::LIT && x.type == "boolean") { if (x.null) push(PO_LIT_NULL); else push(PO_LIT_INT, 0, x.iv); return; }
    if (x.k == Ex::CALL && x.name == "COALESCE") { operand(x); return; }
    if (!is_predicate(x)) refuse("partition predicate " + (x.k == Ex::CALL ? x.name : std::string("operand")) +
                                 " is not supported by this engine build");
    const std::string& n = x.name;
    const auto& c = x.args;
    if (n == "ALWAYS_TRUE" || n == "ALWAYS_FALSE") { push(PO_LIT_INT, 0, n == "ALWAYS_TRUE"); return; }
    if (n == "STARTS_WITH" || n == "LIKE") { string_pred(x); return; }
    if (n == "AND" || n == "OR") {
      if (c.size() != 2) refuse(n + " takes two predicates");
      const bool swap = need(c[1]) > need(c[0]);     // the deeper operand first (Sethi-Ullman order)
      pred(c[swap ? 1 : 0]);
      pred(c[swap ? 0 : 1]);
      push(n == "AND" ? PO_AND : PO_OR);
      return;
    }
    if (n == "NOT") { if (c.size() != 1) refuse("NOT takes one predicate"); pred(c[0]); push(PO_NOT); return; }
    if (n == "IS_NULL" || n == "IS_NOT_NULL") {
      if (c.size() != 1) refuse(n + " takes one operand");
      operand(c[0]);
      push(n == "IS_NULL" ? PO_ISNULL : PO_ISNOTNULL);
      return;
    }
    if (c.size() != 2) refuse(n + " takes two operands");
    const std::string ta = type_of(c[0]), tb = type_of(c[1]);
    if (is_float(ta) || is_float(tb)) { float_cmp(n, c[0], c[1]); return; }
    if (!comparable(ta, tb)) unsupported_expr(n, ta, tb);
    const std::string ka = operand(c[0]), kb = operand(c[1]);
    if (!ka.empty() && !kb.empty() && ka != kb) refuse("comparison of " + ka + " with " + kb + " is not supported");
    push(n == "<" ? PO_LT : n == "<=" ? PO_LE : n == ">" ? PO_GT : n == ">=" ? PO_GE : n == "=" ? PO_EQ : PO_NSEQ);
  }
  // Two float-typed values with no literal side to plan a threshold from (two columns, two literals):
  // both operands on the stack, compared on the device after the ImplicitCastExpression widening
  // (the wider of the two types; PO_FCMP2 parses each float value exactly to its own type).
  void float_values_cmp(const std::string& n, const Ex& a, const Ex& b) {
    const std::string ta = type_of(a), tb = type_of(b);
    auto form = [&](const Ex& x, const std::string& t) {
      if (!is_float(t) && !is_integral(t)) refuse("comparison of " + ta + " with " + tb + " is not supported");
      if (x.k == Ex::LIT && is_float(t)) {             // IEEE bits as an integer literal
        if (x.null) push(PO_LIT_NULL); else push(PO_LIT_INT, 0, (long long)x.bits);
      } else {
        operand(x);
      }
      return is_integral(t) ? FF_INTEGRAL : t == "float" ? FF_FLOAT : FF_DOUBLE;
    };
    const bool swap = need(b) > need(a);
    int fa, fb;
    if (swap) { fb = form(b, tb); fa = form(a, ta); } else { fa = form(a, ta); fb = form(b, tb); }
    const std::string c = swap ? reverse_cmp(n) : n;
    const int cop = c == "<" ? PO_LT : c == "<=" ? PO_LE : c == ">" ? PO_GT : c == ">=" ? PO_GE : c == "=" ? PO_EQ : PO_NSEQ;
    const bool dbl = ta == "double" || tb == "double";
    push(PO_FCMP2, cop | (int)dbl << 8 | (swap ? fb : fa) << 12 | (swap ? fa : fb) << 16);
  }
  void float_cmp(std::string n, const Ex& l0, const Ex& r0) {
    const Ex* left = &l0;
    const Ex* right = &r0;
    if (left->k == Ex::LIT && right->k != Ex::LIT) { std::swap(left, right); n = reverse_cmp(n); }
    const std::string ct = type_of(*left), lt = type_of(*right);
    if (!comparable(ct, lt)) unsupported_expr(n, ct, lt);
    std::string phys, tt;
    if (!field_ref(*left, &phys, &tt) || right->k != Ex::LIT) { float_values_cmp(n, l0, r0); return; }
    if (!is_float(ct) && !is_integral(ct)) refuse("comparison of " + ct + " with " + lt + " is not supported");
    auto cmp_code = [](const std::string& c) {
      return c == "<" ? PO_LT : c == "<=" ? PO_LE : c == ">" ? PO_GT : c == ">=" ? PO_GE : c == "=" ? PO_EQ : PO_NSEQ;
    };
    if (right->null) { operand(*left); push(PO_LIT_NULL); push(cmp_code(n)); return; }
    const std::string cmp_t = ct == lt ? ct : (up_cast(ct, lt) ? lt : ct);
    const std::string value_fmt = is_float(ct) ? ct : cmp_t;
    const std::string op = n == "IS NOT DISTINCT FROM" ? "=" : n;
    std::vector<Cond> conds;
    RankRun rr;
    if (!plan(op, *right, value_fmt, cmp_t, &conds, &rr)) refuse("float literal narrowed");
    int terms = 0;
    if (n == "IS NOT DISTINCT FROM") { operand(*left); push(PO_ISNOTNULL); terms++; }   // a null column: false
    if (!is_float(ct)) {
      long long a, b;
      std::vector<std::pair<int, long long>> parts;
      if (!integral_bounds(conds, &a, &b)) parts.push_back({PO_LT, LLONG_MIN});
      else {
        if (a > LLONG_MIN) parts.push_back({PO_GE, a});
        if (b < LLONG_MAX) parts.push_back({PO_LE, b});
        if (parts.empty()) parts.push_back({PO_GE, LLONG_MIN});
      }
      for (auto& p : parts) {
        operand(*left);
        push(PO_LIT_INT, 0, p.second);
        push(p.first);
        if (++terms > 1) push(PO_AND);
      }
      return;
    }
    const int flags = ((int)rr.nan << 4) | ((int)rr.pinf << 5) | ((int)rr.ninf << 6);
    for (const Cond& c : conds) {
      operand(*left);
      Op o;
      o.op = PO_FCMP;
      if (c.k == C_ALL || c.k == C_NONE) o.arg = flags | (c.k == C_ALL ? FC_ALL : FC_NONE);
      else {
        o.arg = flags | (c.k == C_LT ? FC_LT : c.k == C_LE ? FC_LE : c.k == C_GT ? FC_GT : FC_GE);
        o.has_bytes = true;
        o.bytes = decimal_text(c.B);
      }
      ops.push_back(o);
      if (++terms > 1) push(PO_AND);
    }
  }
};

int pt_code(const std::string& t) {
  static const char* names[] = {"long", "integer", "short", "byte", "string", "date", "decimal", "boolean", "float", "double", "timestamp"};
  for (int i = 0; i < 11; i++) if (t == names[i]) return i;
  return -1;
}

// literal bytes into the pool, in op order (after the names)
void finalize_ops(dk_program& P, const std::vector<Op>& ops, bool skipping) {
  P.op.clear(); P.arg.clear(); P.lit.clear();
  for (const Op& o : ops) {
    int32_t arg = o.arg;
    int64_t lit = o.lit;
    if (o.has_bytes) {
      const int64_t off = (int64_t)P.pool.size();
      if (o.op == (skipping ? OP_FCMP : PO_FCMP) || (!skipping && (o.op == PO_STARTS_WITH || o.op == PO_LIKE))) {
        lit = off | ((int64_t)o.bytes.size() << 32);
        P.pool += o.bytes;
        if (o.ranks) {
          int64_t r[2] = {o.r0, o.r1};
          P.pool.append((const char*)r, 16);
        }
      } else {                                       // LIT_STR / LIT_DEC: length in arg, offset in lit
        arg = (int32_t)o.bytes.size();
        lit = off;
        P.pool += o.bytes;
      }
    }
    P.op.push_back(o.op);
    P.arg.push_back(arg);
    P.lit.push_back(lit);
  }
}

int compile_status(const Unsupported& u) { dk::dk_fail(u.msg); return u.code; }

}  // namespace

namespace dk {
// the leaves of a (pruned stats) schema as the path table of a program with no ops: what
// dk_json_parse extracts from each row (JsonHandler.parseJson's output schema)
int schema_program(const char* schema_json, dk_program* out) {
  JV sj;
  std::string err;
  if (!parse_json(schema_json, sj, err)) return dk_fail("dk_json_parse: schema: " + err);
  std::vector<std::pair<Path, std::string>> leaves;
  Path prefix;
  if (sj.t != JV::OBJ || !walk_schema(sj, prefix, leaves, err)) return dk_fail("dk_json_parse: " + (err.empty() ? "bad schema" : err));
  *out = dk_program();
  out->kind = DK_PROGRAM_SKIPPING;
  for (auto& l : leaves) {
    const int code = sk_type_code(l.second);
    if (code < 0) return dk_fail("dk_json_parse: " + l.second + " fields are not supported by this engine (stats schemas only)");
    out->path_type.push_back(code);
    out->paths.push_back(l.first);
    out->path_comp.push_back((int32_t)out->comp_off.size());
    for (auto& c : l.first) {
      out->comp_off.push_back((int32_t)out->pool.size());
      out->comp_len.push_back((int32_t)c.size());
      out->pool += c;
    }
  }
  out->path_comp.push_back((int32_t)out->comp_off.size());
  return 0;
}

std::string program_image(const dk_program& p, int64_t offs[8]) {
  std::string img;
  auto put = [&](const void* d, size_t n) {
    while (img.size() % 8) img += '\0';
    const int64_t at = (int64_t)img.size();
    img.append((const char*)d, n);
    return at;
  };
  if (p.kind == DK_PROGRAM_SKIPPING) {
    offs[0] = put(p.path_type.data(), p.path_type.size() * 4);
    offs[1] = put(p.path_comp.data(), p.path_comp.size() * 4);
    offs[2] = put(p.comp_off.data(), p.comp_off.size() * 4);
    offs[3] = put(p.comp_len.data(), p.comp_len.size() * 4);
  } else {
    offs[0] = put(p.field_type.data(), p.field_type.size() * 4);
    offs[1] = put(p.name_off.data(), p.name_off.size() * 4);
    offs[2] = put(p.name_len.data(), p.name_len.size() * 4);
    offs[3] = offs[2];
  }
  offs[4] = put(p.op.data(), p.op.size() * 4);
  offs[5] = put(p.arg.data(), p.arg.size() * 4);
  offs[6] = put(p.lit.data(), p.lit.size() * 8);
  offs[7] = put(p.pool.data(), p.pool.size());
  img.append(64, '\0');                              // slack for word-wise reads of the pool
  return img;
}
}  // namespace dk

extern "C" int dk_skip_compile(const char* stats_schema_json, const char* predicate_json, dk_program** out) {
  if (!out) return dk::dk_fail("dk_skip_compile: null out");
  *out = nullptr;
  JV sj, pj;
  std::string err;
  if (!parse_json(stats_schema_json, sj, err)) return dk::dk_fail("dk_skip_compile: stats schema: " + err);
  if (!parse_json(predicate_json, pj, err)) return dk::dk_fail("dk_skip_compile: predicate: " + err);
  std::vector<std::pair<Path, std::string>> leaves;
  Path prefix;
  if (sj.t != JV::OBJ || !walk_schema(sj, prefix, leaves, err)) return dk::dk_fail("dk_skip_compile: " + (err.empty() ? "bad schema" : err));
  Ex root;
  if (!to_expr(pj, root, err)) return dk::dk_fail("dk_skip_compile: " + err);
  std::unique_ptr<dk_program> P(new dk_program());
  P->kind = DK_PROGRAM_SKIPPING;
  try {
    SkipCompiler C;
    for (auto& l : leaves) C.schema[l.first] = l.second;
    const Ex* pred = unwrap_skipping(root);
    C.check(*pred);
    C.collect(*pred);
    C.emit(*pred);
    if (depth_of(C.ops, true) > kMaxStack) {           // re-associate AND / OR chains
      C.ops.clear();
      const Ex b = rebalance(*pred);
      C.emit(b);
      if (depth_of(C.ops, true) > kMaxStack) refuse("data skipping filter nests deeper than the device stack");
    }
    for (auto& p : C.paths) {
      const int code = sk_type_code(C.schema[p]);
      if (code < 0) refuse("data skipping on " + C.schema[p] + " stats is not supported");
      P->path_type.push_back(code);
      P->paths.push_back(p);
      P->path_comp.push_back((int32_t)P->comp_off.size());
      for (auto& s : p) {
        P->comp_off.push_back((int32_t)P->pool.size());
        P->comp_len.push_back((int32_t)s.size());
        P->pool += s;
      }
    }
    P->path_comp.push_back((int32_t)P->comp_off.size());
    finalize_ops(*P, C.ops, true);
    P->stack = depth_of(C.ops, true);
  } catch (const Unsupported& u) {
    return compile_status(u);
  } catch (const std::exception& e) {
    return dk::dk_fail(std::string("dk_skip_compile: ") + e.what());
  }
  if (P->pool.size() > (size_t)INT32_MAX) return dk::dk_fail("dk_skip_compile: literals exceed 2 GiB");
  *out = P.release();
  return 0;
}

extern "C" int dk_part_compile(const char* predicate_json, dk_program** out) {
  if (!out) return dk::dk_fail("dk_part_compile: null out");
  *out = nullptr;
  JV pj;
  std::string err;
  if (!parse_json(predicate_json, pj, err)) return dk::dk_fail("dk_part_compile: predicate: " + err);
  Ex root;
  if (!to_expr(pj, root, err)) return dk::dk_fail("dk_part_compile: " + err);
  std::unique_ptr<dk_program> P(new dk_program());
  P->kind = DK_PROGRAM_PARTITION;
  try {
    PartCompiler C;
    C.pred(root);
    if (depth_of(C.ops, false) > kMaxStack) {
      C.ops.clear();
      C.used.clear();
      C.types_full.clear();
      const Ex b = rebalance(root);
      C.pred(b);
      if (depth_of(C.ops, false) > kMaxStack) refuse("partition filter nests deeper than the device stack");
    }
    for (auto& u : C.used) {
      P->field_type.push_back(pt_code(u.second));
      P->fields.push_back(u.first);
      P->name_off.push_back((int32_t)P->pool.size());
      P->name_len.push_back((int32_t)u.first.size());
      P->pool += u.first;
    }
    finalize_ops(*P, C.ops, false);
    P->stack = depth_of(C.ops, false);
  } catch (const Unsupported& u) {
    return compile_status(u);
  } catch (const std::exception& e) {
    return dk::dk_fail(std::string("dk_part_compile: ") + e.what());
  }
  if (P->pool.size() > (size_t)INT32_MAX) return dk::dk_fail("dk_part_compile: literals exceed 2 GiB");
  *out = P.release();
  return 0;
}

extern "C" void dk_program_free(dk_program* p) { delete p; }

// JSON description of a compiled program: {"kind", "paths" | "fields", "stack", "ops": [[op, arg, lit], ...],
// "pool": hex}; the skipping paths are what a caller projects as add.stats_parsed.<path>
extern "C" int64_t dk_program_describe(const dk_program* p, char* buf, int64_t cap) {
  if (!p) return -1;
  std::string s = "{\"kind\":" + std::to_string(p->kind) + ",\"stack\":" + std::to_string(p->stack);
  auto q = [](const std::string& x) {
    std::string o = "\"";
    for (unsigned char c : x) {
      if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
      else if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
      else o += (char)c;
    }
    return o + "\"";
  };
  if (p->kind == DK_PROGRAM_SKIPPING) {
    s += ",\"paths\":[";
    for (size_t i = 0; i < p->paths.size(); i++) {
      s += (i ? "," : "") + std::string("{\"type\":") + std::to_string(p->path_type[i]) + ",\"path\":[";
      for (size_t k = 0; k < p->paths[i].size(); k++) s += (k ? "," : "") + q(p->paths[i][k]);
      s += "]}";
    }
    s += "]";
  } else {
    s += ",\"fields\":[";
    for (size_t i = 0; i < p->fields.size(); i++)
      s += (i ? "," : "") + std::string("{\"type\":") + std::to_string(p->field_type[i]) + ",\"name\":" + q(p->fields[i]) + "}";
    s += "]";
  }
  s += ",\"ops\":[";
  for (size_t i = 0; i < p->op.size(); i++)
    s += (i ? "," : "") + std::string("[") + std::to_string(p->op[i]) + "," + std::to_string(p->arg[i]) + "," +
         std::to_string(p->lit[i]) + "]";
  s += "],\"pool\":\"";
  static const char* hx = "0123456789abcdef";
  for (unsigned char c : p->pool) { s += hx[c >> 4]; s += hx[c & 15]; }
  s += "\"}";
  if (buf && cap > 0) {
    const int64_t n = (int64_t)s.size() < cap - 1 ? (int64_t)s.size() : cap - 1;
    memcpy(buf, s.data(), (size_t)n);
    buf[n] = 0;
  }
  return (int64_t)s.size();
}
