/*
 * dk_skip — CPU ORACLE (test infrastructure only): a C fast path for oracle/skipping.py's `keep`
 * over integral stats, so that the full-size C4 parity check (50M rows, `id > 25000000`) and its
 * CPU baseline finish in seconds instead of hours of per-row Python.
 *
 * Only tests/ and bench.py's cpu_baseline leg load it (via oracle/ref.py). The product never does.
 *
 * What it restates (the same rules as oracle/skipping.py, which is the pinned restatement):
 *   DefaultJsonHandler.parseJson   kernel-defaults/.../engine/DefaultJsonHandler.java:60-76,193-200
 *       Jackson readTree: leading whitespace, the root must be an object, trailing content ignored,
 *       the last duplicate key wins (ObjectNode.set)
 *   DefaultJsonRow.decodeElement   kernel-defaults/.../internal/data/DefaultJsonRow.java:136-270
 *       long / integer: an integral JSON number in range; short / byte: any number whose exact
 *       value is an integer in range; JSON null or a missing field = null
 *   DefaultExpressionEvaluator     comparators null when either side is null, Kleene AND / OR
 *   ScanImpl.applyDataSkipping     kernel-api/.../internal/ScanImpl.java:304-352
 *       the row stays iff COALESCE(predicate, true)
 *
 * It decides a row only when everything is clean. Every row it is not sure about (anything Python's
 * json module or the decode rules would reject, escaped keys, exponents beyond +-400, nesting
 * deeper than 64) is marked `defer` and evaluated by oracle/skipping.py itself, which also raises
 * the reference's decode errors. tests/test_oracle_skip_fast.py checks it row for row against
 * oracle/skipping.keep.
 */
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

enum { T_LONG = 0, T_INT = 1, T_SHORT = 2, T_BYTE = 3 };
enum { OP_STAT = 1, OP_LIT = 2, OP_LT = 3, OP_LE = 4, OP_GT = 5, OP_GE = 6, OP_EQ = 7, OP_AND = 8, OP_OR = 9 };
enum { K_MISSING = 0, K_NULL, K_INT, K_DEC, K_OTHER, K_NOTOBJ };   /* leaf / path states */

#define MAXP 16
#define MAXC 8
#define MAXDEPTH 64

typedef struct {
    int type, ncomp;
    const char* comp[MAXC];
    int clen[MAXC];
} SPath;

typedef struct {
    int kind;
    const char *b, *e;          /* the leaf token */
} SVal;

typedef struct {
    const char *p, *end;
    int bad;                    /* 1: not sure / invalid -> defer */
    const SPath* paths;
    int np;
    SVal* vals;
} Parser;

static void ws(Parser* P) {
    while (P->p < P->end && (*P->p == ' ' || *P->p == '\t' || *P->p == '\n' || *P->p == '\r')) P->p++;
}

static int hexd(char c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
}

/* a JSON string starting at '"'; sets *esc when it holds an escape. Python's json (strict) rejects
 * control characters < 0x20 inside strings and unknown escapes. */
static void str_tok(Parser* P, const char** sb, const char** se, int* esc) {
    P->p++;
    *sb = P->p;
    *esc = 0;
    while (P->p < P->end) {
        unsigned char c = (unsigned char)*P->p;
        if (c == '"') { *se = P->p; P->p++; return; }
        if (c < 0x20) { P->bad = 1; return; }
        if (c == '\\') {
            *esc = 1;
            if (P->p + 1 >= P->end) { P->bad = 1; return; }
            char n = P->p[1];
            if (n == 'u') {
                if (P->p + 6 > P->end || !hexd(P->p[2]) || !hexd(P->p[3]) || !hexd(P->p[4]) || !hexd(P->p[5])) {
                    P->bad = 1; return;
                }
                P->p += 6;
                continue;
            }
            if (!strchr("\"\\/bfnrt", n) || n == 0) { P->bad = 1; return; }
            P->p += 2;
            continue;
        }
        P->p++;
    }
    P->bad = 1;
}

/* -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][-+]?[0-9]+)?  (Python json's NUMBER_RE) */
static int num_tok(Parser* P) {
    const char* s = P->p;
    int dec = 0;
    if (s < P->end && *s == '-') s++;
    if (s >= P->end) { P->bad = 1; return K_OTHER; }
    if (*s == '0') s++;
    else if (*s >= '1' && *s <= '9') { while (s < P->end && *s >= '0' && *s <= '9') s++; }
    else { P->bad = 1; return K_OTHER; }
    if (s + 1 < P->end && *s == '.' && s[1] >= '0' && s[1] <= '9') {
        dec = 1; s++;
        while (s < P->end && *s >= '0' && *s <= '9') s++;
    }
    if (s < P->end && (*s == 'e' || *s == 'E')) {
        const char* t = s + 1;
        if (t < P->end && (*t == '+' || *t == '-')) t++;
        if (t < P->end && *t >= '0' && *t <= '9') {
            dec = 1;
            while (t < P->end && *t >= '0' && *t <= '9') t++;
            s = t;
        }
    }
    P->p = s;
    return dec ? K_DEC : K_INT;
}

static void value(Parser* P, int depth, const int* cand, int nc);

/* the object at P->p ('{'); cand = the paths whose components 0..depth-1 led here */
static void object(Parser* P, int depth, const int* cand, int nc) {
    if (depth >= MAXDEPTH) { P->bad = 1; return; }
    P->p++;
    ws(P);
    if (P->p < P->end && *P->p == '}') { P->p++; return; }
    for (;;) {
        ws(P);
        if (P->p >= P->end || *P->p != '"') { P->bad = 1; return; }
        const char *kb, *ke;
        int esc;
        str_tok(P, &kb, &ke, &esc);
        if (P->bad) return;
        ws(P);
        if (P->p >= P->end || *P->p != ':') { P->bad = 1; return; }
        P->p++;
        ws(P);
        int sub[MAXP], ns = 0;
        for (int i = 0; i < nc; i++) {
            const SPath* sp = &P->paths[cand[i]];
            if (depth < sp->ncomp && sp->clen[depth] == (int)(ke - kb) && !memcmp(sp->comp[depth], kb, ke - kb))
                sub[ns++] = cand[i];
        }
        if (esc && nc) { P->bad = 1; return; }          /* escaped keys: left to the Python restatement */
        /* a later duplicate key replaces everything under it (ObjectNode.set) */
        for (int i = 0; i < ns; i++) P->vals[sub[i]].kind = K_MISSING;
        value(P, depth + 1, sub, ns);
        if (P->bad) return;
        ws(P);
        if (P->p < P->end && *P->p == ',') { P->p++; continue; }
        if (P->p < P->end && *P->p == '}') { P->p++; return; }
        P->bad = 1;
        return;
    }
}

static void array(Parser* P, int depth) {
    if (depth >= MAXDEPTH) { P->bad = 1; return; }
    P->p++;
    ws(P);
    if (P->p < P->end && *P->p == ']') { P->p++; return; }
    for (;;) {
        ws(P);
        value(P, depth + 1, NULL, 0);
        if (P->bad) return;
        ws(P);
        if (P->p < P->end && *P->p == ',') { P->p++; continue; }
        if (P->p < P->end && *P->p == ']') { P->p++; return; }
        P->bad = 1;
        return;
    }
}

static int lit(Parser* P, const char* w) {
    size_t n = strlen(w);
    if ((size_t)(P->end - P->p) >= n && !memcmp(P->p, w, n)) { P->p += n; return 1; }
    return 0;
}

/* a value; cand = paths whose component `depth-1` is this value's key */
static void value(Parser* P, int depth, const int* cand, int nc) {
    if (P->p >= P->end) { P->bad = 1; return; }
    const char* b = P->p;
    int kind;
    char c = *P->p;
    if (c == '{') {
        int inner[MAXP], ni = 0;
        for (int i = 0; i < nc; i++) {
            if (P->paths[cand[i]].ncomp > depth) inner[ni++] = cand[i];
            else P->vals[cand[i]].kind = K_OTHER;       /* an object where a leaf value is wanted */
        }
        object(P, depth, inner, ni);
        return;
    }
    if (c == '[') { array(P, depth); kind = K_OTHER; }
    else if (c == '"') { const char *sb, *se; int esc; str_tok(P, &sb, &se, &esc); kind = K_OTHER; }
    else if (c == '-' || (c >= '0' && c <= '9')) kind = num_tok(P);
    else if (lit(P, "true") || lit(P, "false")) kind = K_OTHER;
    else if (lit(P, "null")) kind = K_NULL;
    else { P->bad = 1; return; }
    if (P->bad) return;
    for (int i = 0; i < nc; i++) {
        SVal* v = &P->vals[cand[i]];
        if (P->paths[cand[i]].ncomp > depth)             /* an intermediate component */
            v->kind = kind == K_NULL ? K_NULL : K_NOTOBJ;
        else { v->kind = kind; v->b = b; v->e = P->p; }
    }
}

/* exact integral value of a clean number token; 0 = not an integer in [lo, hi] or unsure */
static int integral(const char* b, const char* e, int dec, int64_t lo, int64_t hi, int64_t* out) {
    int neg = 0;
    if (*b == '-') { neg = 1; b++; }
    char dig[64];
    int nd = 0, frac = 0, in_frac = 0;
    long exp = 0;
    const char* s = b;
    for (; s < e && *s != 'e' && *s != 'E'; s++) {
        if (*s == '.') { in_frac = 1; continue; }
        if (nd == 0 && *s == '0') { if (in_frac) frac++; continue; }   /* leading zeros */
        if (nd >= 60) return 0;
        dig[nd++] = *s;
        if (in_frac) frac++;
    }
    if (s < e) {
        if (!dec) return 0;
        s++;
        int eneg = 0;
        if (*s == '+' || *s == '-') eneg = *s++ == '-';
        for (; s < e; s++) {
            exp = exp * 10 + (*s - '0');
            if (exp > 400) return 0;
        }
        if (eneg) exp = -exp;
    }
    if (nd == 0) { *out = 0; return lo <= 0 && 0 <= hi; }
    /* value = dig * 10^(exp - frac), dig without leading zeros; move trailing zeros to the exponent */
    long e10 = exp - frac;
    while (nd > 0 && dig[nd - 1] == '0') { nd--; e10++; }
    if (e10 < 0) return 0;                      /* not integral */
    if (nd + e10 > 18) return 0;                /* beyond every integral range here: unsure -> defer */
    int64_t v = 0;
    for (int i = 0; i < nd; i++) v = v * 10 + (dig[i] - '0');
    for (long i = 0; i < e10; i++) v *= 10;
    if (neg) v = -v;
    if (v < lo || v > hi) return 0;
    *out = v;
    return 1;
}

static const int64_t LO[4] = {INT64_MIN, -2147483648LL, -32768, -128};
static const int64_t HI[4] = {INT64_MAX, 2147483647LL, 32767, 127};

/* 19-digit tokens may still fit a long: exact check */
static int long_token(const char* b, const char* e, int64_t* out) {
    int neg = *b == '-';
    const char* s = b + neg;
    if (e - s > 19) return 0;
    uint64_t v = 0;
    for (; s < e; s++) {
        uint64_t d = (uint64_t)(*s - '0');
        if (v > (UINT64_MAX - d) / 10) return 0;
        v = v * 10 + d;
    }
    if (!neg && v > (uint64_t)INT64_MAX) return 0;
    if (neg && v > (uint64_t)INT64_MAX + 1) return 0;
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 1;
}

/* 1 keep, 0 drop, -1 defer */
static int eval_row(const char* s, int64_t n, const SPath* paths, int np, const int64_t* prog, int nops) {
    SVal vals[MAXP];
    memset(vals, 0, sizeof vals);
    Parser P = {s, s + n, 0, paths, np, vals};
    ws(&P);
    if (P.p >= P.end || *P.p != '{') return -1;
    int cand[MAXP];
    for (int i = 0; i < np; i++) cand[i] = i;
    object(&P, 0, cand, np);
    if (P.bad) return -1;
    /* decode every referenced path (decode_stats decodes them all before evaluating) */
    int isnull[MAXP];
    int64_t iv[MAXP];
    for (int i = 0; i < np; i++) {
        SVal* v = &vals[i];
        int t = paths[i].type;
        isnull[i] = 0;
        if (v->kind == K_MISSING || v->kind == K_NULL) { isnull[i] = 1; continue; }
        if (v->kind == K_INT) {
            int64_t x;
            if (!long_token(v->b, v->e, &x) || x < LO[t] || x > HI[t]) return -1;
            iv[i] = x;
            continue;
        }
        if (v->kind == K_DEC && (t == T_SHORT || t == T_BYTE)) {
            if (!integral(v->b, v->e, 1, LO[t], HI[t], &iv[i])) return -1;
            continue;
        }
        return -1;                              /* a decode error in the reference: Python raises it */
    }
    /* stack: 0 false, 1 true, 2 null for booleans; ints carry their value */
    int64_t sv[64];
    int sk[64];                                 /* 0 bool, 1 int, 2 null */
    int sp = 0;
    for (int k = 0; k < nops; k++) {
        int64_t op = prog[2 * k], a = prog[2 * k + 1];
        if (sp >= 62) return -1;
        switch (op) {
        case OP_STAT:
            if (a < 0 || a >= np) return -1;
            if (isnull[a]) { sk[sp] = 2; sv[sp] = 0; }
            else { sk[sp] = 1; sv[sp] = iv[a]; }
            sp++;
            break;
        case OP_LIT: sk[sp] = 1; sv[sp] = a; sp++; break;
        case OP_LT: case OP_LE: case OP_GT: case OP_GE: case OP_EQ: {
            if (sp < 2) return -1;
            int64_t x = sv[sp - 2], y = sv[sp - 1];
            int null = sk[sp - 2] == 2 || sk[sp - 1] == 2;
            sp -= 2;
            int r = op == OP_LT ? x < y : op == OP_LE ? x <= y : op == OP_GT ? x > y : op == OP_GE ? x >= y : x == y;
            sk[sp] = null ? 2 : 0;
            sv[sp] = null ? 2 : r;
            sp++;
            break;
        }
        case OP_AND: case OP_OR: {
            if (sp < 2) return -1;
            int64_t x = sv[sp - 2], y = sv[sp - 1];   /* 0 / 1 / 2 */
            sp -= 2;
            int64_t r;
            if (op == OP_AND) r = (x == 0 || y == 0) ? 0 : (x == 1 && y == 1) ? 1 : 2;
            else r = (x == 1 || y == 1) ? 1 : (x == 0 && y == 0) ? 0 : 2;
            sk[sp] = r == 2 ? 2 : 0;
            sv[sp] = r;
            sp++;
            break;
        }
        default:
            return -1;
        }
    }
    if (sp != 1) return -1;
    return sv[0] != 0;                          /* COALESCE(pred, true): only FALSE drops the row */
}

/* Paths blob: per path {u8 type, u8 ncomp, per component {u16 len, bytes}}. prog: (op, arg) int64
 * pairs in postfix order. For every row with sel[r] != 0: the row's add.stats (null when
 * row_def[r] < max_def: kept) is evaluated; sel[r] = 0 when the predicate is FALSE; defer[r] = 1
 * when the row is left to the Python restatement. Returns the number of deferred rows, or -1 on a
 * malformed program. */
EXPORT int64_t dkr_skip_eval(const uint8_t* chars, const int64_t* offs, const uint8_t* row_def, int max_def,
                             uint8_t* sel, uint8_t* defer, int64_t n_rows, const uint8_t* blob, int64_t blob_len,
                             int np, const int64_t* prog, int nops) {
    SPath paths[MAXP];
    if (np < 1 || np > MAXP) return -1;
    int64_t q = 0;
    for (int i = 0; i < np; i++) {
        if (q + 2 > blob_len) return -1;
        paths[i].type = blob[q];
        paths[i].ncomp = blob[q + 1];
        q += 2;
        if (paths[i].type < 0 || paths[i].type > 3 || paths[i].ncomp < 1 || paths[i].ncomp > MAXC) return -1;
        for (int c = 0; c < paths[i].ncomp; c++) {
            if (q + 2 > blob_len) return -1;
            int len = blob[q] | (blob[q + 1] << 8);
            q += 2;
            if (q + len > blob_len) return -1;
            paths[i].comp[c] = (const char*)blob + q;
            paths[i].clen[c] = len;
            q += len;
        }
    }
    int64_t nd = 0;
    for (int64_t r = 0; r < n_rows; r++) {
        defer[r] = 0;
        if (!sel[r] || row_def[r] < max_def) continue;
        int k = eval_row((const char*)chars + offs[r], offs[r + 1] - offs[r], paths, np, prog, nops);
        if (k < 0) { defer[r] = 1; nd++; }
        else if (k == 0) sel[r] = 0;
    }
    return nd;
}
