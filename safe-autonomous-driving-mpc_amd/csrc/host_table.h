// host_table.h -- host-only parts of libmpcqp (no HIP): the trajectory JSON reader and the build of the
// reference-signal table that mpc_create copies to the device.  Kept free of device code so that a CPU
// test target compiles exactly this file with -fsanitize=address,undefined (tests/asan/).
//
//   read_trajectory_json_text  replaces the json.load of TrajectoryLoader.__init__
//                              (medinammartin3/Safe-Autonomous-Driving-MPC trajectory_loader.py:13-24)
//   build_host_table           the strict-monotone s fix (trajectory_loader.py:26-30), the interp1d columns
//                              (:64-84, u over s[:min(T, Tu)]), the global reference line (:32-62) and the
//                              bucket index of the s column used by the device lookups (seg_t)
#ifndef MPCQP_HOST_TABLE_H
#define MPCQP_HOST_TABLE_H

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace mpcqp_host {

// ---------------------------------------------------------------------------------------------
// trajectory JSON: {"X": [[s,d,o,k,v], ...], "U": [[u1,u2], ...], ...}; other keys are skipped.
// Semantics follow Python's json.load as the reference uses it: a repeated key keeps its LAST value,
// trailing data after the top-level object is an error, nesting deeper than MAX_DEPTH is refused.
// ---------------------------------------------------------------------------------------------
struct JsonReader {
    static constexpr int MAX_DEPTH = 256;
    const char* p;
    const char* end;     // *end is '\0' (std::string storage), so strtod never reads past it
    std::string err;

    void ws() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
    bool expect(char ch) {
        ws();
        if (p < end && *p == ch) { ++p; return true; }
        err = std::string("expected '") + ch + "'";
        return false;
    }
    static int hexval(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    bool string(std::string* out) {
        if (!expect('"')) return false;
        std::string r;
        while (p < end && *p != '"') {
            if (*p != '\\') { r.push_back(*p++); continue; }
            if (p + 1 >= end) break;
            const char e = p[1];
            p += 2;
            switch (e) {
                case 'n': r.push_back('\n'); break;
                case 't': r.push_back('\t'); break;
                case 'r': r.push_back('\r'); break;
                case 'b': r.push_back('\b'); break;
                case 'f': r.push_back('\f'); break;
                case 'u': {          // \uXXXX: BMP code point as UTF-8 (keys such as "X" == "X")
                    if (end - p < 4) { err = "bad \\u escape"; return false; }
                    unsigned cp = 0;
                    for (int i = 0; i < 4; ++i) {
                        const int h = hexval(p[i]);
                        if (h < 0) { err = "bad \\u escape"; return false; }
                        cp = cp * 16 + (unsigned)h;
                    }
                    p += 4;
                    if (cp < 0x80) {
                        r.push_back((char)cp);
                    } else if (cp < 0x800) {
                        r.push_back((char)(0xC0 | (cp >> 6)));
                        r.push_back((char)(0x80 | (cp & 0x3F)));
                    } else {
                        r.push_back((char)(0xE0 | (cp >> 12)));
                        r.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
                        r.push_back((char)(0x80 | (cp & 0x3F)));
                    }
                    break;
                }
                default: r.push_back(e);  // \" \\ \/
            }
        }
        if (p >= end) { err = "unterminated string"; return false; }
        ++p;
        if (out) *out = r;
        return true;
    }
    bool number(double* out) {
        ws();
        // JSON numbers only (json.load also takes NaN / Infinity / -Infinity); strtod alone would also
        // accept "inf", "nan" and hex floats
        const char* q = p;
        if (q < end && *q == '-') ++q;
        if (end - q >= 8 && !std::strncmp(q, "Infinity", 8)) {
            *out = (*p == '-') ? -INFINITY : INFINITY;
            p = q + 8;
            return true;
        }
        if (q == p && end - q >= 3 && !std::strncmp(q, "NaN", 3)) {
            *out = NAN;
            p = q + 3;
            return true;
        }
        if (q >= end || *q < '0' || *q > '9') { err = "expected a number"; return false; }
        char* e = nullptr;
        const double v = std::strtod(p, &e);
        if (e == p || e > end) { err = "expected a number"; return false; }
        for (const char* c = p; c < e; ++c)
            if (*c == 'x' || *c == 'X' || *c == 'p' || *c == 'P') { err = "expected a number"; return false; }
        p = e;
        *out = v;
        return true;
    }
    bool skip(int depth = 0) {   // any value
        ws();
        if (p >= end) { err = "unexpected end"; return false; }
        if (depth > MAX_DEPTH) { err = "nesting too deep"; return false; }
        if (*p == '"') return string(nullptr);
        if (*p == '{' || *p == '[') {
            const char open = *p, close = open == '{' ? '}' : ']';
            ++p;
            ws();
            if (p < end && *p == close) { ++p; return true; }
            while (true) {
                if (open == '{') { if (!string(nullptr) || !expect(':')) return false; }
                if (!skip(depth + 1)) return false;
                ws();
                if (p < end && *p == ',') { ++p; continue; }
                return expect(close);
            }
        }
        if (end - p >= 4 && !std::strncmp(p, "true", 4)) { p += 4; return true; }
        if (end - p >= 5 && !std::strncmp(p, "false", 5)) { p += 5; return true; }
        if (end - p >= 4 && !std::strncmp(p, "null", 4)) { p += 4; return true; }
        double v;
        return number(&v);
    }
    // [[a, b, ...], ...] with rows of exactly `width` numbers; replaces *out (last key wins)
    bool matrix(int width, std::vector<double>* out, int* rows) {
        out->clear();
        *rows = 0;
        if (!expect('[')) return false;
        ws();
        if (p < end && *p == ']') { ++p; return true; }
        while (true) {
            if (!expect('[')) return false;
            for (int j = 0; j < width; ++j) {
                double v;
                if (!number(&v)) return false;
                out->push_back(v);
                if (j + 1 < width && !expect(',')) {
                    err = "row of the wrong width (expected " + std::to_string(width) + " numbers)";
                    return false;
                }
            }
            if (!expect(']')) {
                err = "row of the wrong width (expected " + std::to_string(width) + " numbers)";
                return false;
            }
            ++*rows;
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            return expect(']');
        }
    }
};

// Parse the text of a trajectory JSON.  On success X holds T x 5 and U holds Tu x 2 row-major doubles
// (exactly T*5 and Tu*2 values); on failure returns false with `err` set (byte offset included).
inline bool read_trajectory_json_text(const std::string& text, std::vector<double>& X, int& T,
                                      std::vector<double>& U, int& Tu, std::string& err) {
    JsonReader r{text.data(), text.data() + text.size(), ""};
    X.clear();
    U.clear();
    int tx = -1, tu = -1;
    bool ok = r.expect('{');
    r.ws();
    if (ok && r.p < r.end && *r.p == '}') ok = false, r.err = "empty object";
    while (ok) {
        std::string key;
        ok = r.string(&key) && r.expect(':');
        if (!ok) break;
        if (key == "X") ok = r.matrix(5, &X, &tx);
        else if (key == "U") ok = r.matrix(2, &U, &tu);
        else ok = r.skip(1);
        if (!ok) break;
        r.ws();
        if (r.p < r.end && *r.p == ',') { ++r.p; continue; }
        ok = r.expect('}');
        break;
    }
    if (ok) {
        r.ws();
        if (r.p != r.end) ok = false, r.err = "extra data after the top-level object";
    }
    if (!ok) {
        err = "trajectory JSON: " + r.err + " at byte " + std::to_string((long)(r.p - text.data()));
        return false;
    }
    if (tx < 0 || tu < 0) {
        err = "trajectory JSON: missing 'X' or 'U'";
        return false;
    }
    T = tx;
    Tu = tu;
    return true;
}

// ---------------------------------------------------------------------------------------------
// the device table, built on the host.  One buffer of doubles:
//   s, d, o, k, v [T] | u1, u2 [tu] | gx, gy, gpsi [T] | bucket index (ints) [nb + 1]
// with tu = min(T, Tu) (trajectory_loader.py:73-75) and nb = 4 (T - 1) uniform buckets of the s range,
// bidx[g] = lower_bound(s, s0 + g h).
// ---------------------------------------------------------------------------------------------
struct HostTable {
    std::vector<double> buf;
    int T = 0, tu = 0, nb = 0;
    double smax = 0.0, s0 = 0.0, ibh = 0.0;
    double last[5] = {0, 0, 0, 0, 0};
    size_t off_bidx = 0;      // offset of the bucket index, in doubles
};

inline bool build_host_table(const double* X, int T, const double* U, int Tu, HostTable& h) {
    if (!X || !U || T < 2 || Tu < 2) return false;
    const int tu = Tu < T ? Tu : T;
    const int nb = 4 * (T - 1);
    h.off_bidx = (size_t)8 * T + 2 * (size_t)tu;
    h.buf.assign(h.off_bidx + (size_t)(nb + 2) / 2, 0.0);
    double* s = h.buf.data();
    for (int i = 0; i < T; ++i) {
        double si = X[5 * (size_t)i];
        if (i > 0 && si <= s[i - 1]) si = s[i - 1] + 1e-5;   // trajectory_loader.py:28-30
        s[i] = si;
        h.buf[T + i] = X[5 * (size_t)i + 1];
        h.buf[2 * (size_t)T + i] = X[5 * (size_t)i + 2];
        h.buf[3 * (size_t)T + i] = X[5 * (size_t)i + 3];
        h.buf[4 * (size_t)T + i] = X[5 * (size_t)i + 4];
    }
    for (int i = 0; i < tu; ++i) {
        h.buf[5 * (size_t)T + i] = U[2 * (size_t)i];
        h.buf[5 * (size_t)T + tu + i] = U[2 * (size_t)i + 1];
    }
    // global pose of the reference line: heading integrates X[i-1,3] over ds, position the mean heading
    // of each step (trajectory_loader.py:38-58; host libm, as numpy)
    double* gx = h.buf.data() + 5 * (size_t)T + 2 * (size_t)tu;
    double* gy = gx + T;
    double* gpsi = gy + T;
    gx[0] = gy[0] = gpsi[0] = 0.0;
    for (int i = 1; i < T; ++i) {
        const double ds = s[i] - s[i - 1];
        const double psi_old = gpsi[i - 1];
        const double psi_new = psi_old + X[5 * (size_t)(i - 1) + 3] * ds;
        const double psi_avg = (psi_old + psi_new) / 2.0;
        gpsi[i] = psi_new;
        gx[i] = gx[i - 1] + std::cos(psi_avg) * ds;
        gy[i] = gy[i - 1] + std::sin(psi_avg) * ds;
    }
    int* bidx = reinterpret_cast<int*>(h.buf.data() + h.off_bidx);
    const double bh = (s[T - 1] - s[0]) / nb;
    for (int g = 0, lo = 0; g <= nb; ++g) {
        const double v = s[0] + g * bh;
        while (lo < T && s[lo] < v) ++lo;
        bidx[g] = lo;
    }
    h.T = T;
    h.tu = tu;
    h.nb = nb;
    h.smax = s[T - 1];
    h.s0 = s[0];
    h.ibh = 1.0 / bh;
    for (int j = 0; j < 5; ++j) h.last[j] = X[5 * (size_t)(T - 1) + j];
    return true;
}

// host restatement of the device interval search (seg_t in mpcqp.hip): scipy's searchsorted lower bound
// of v in s[0..T), found by binary search inside the buckets around v's, clamped to [1, n - 1]
inline int seg_host(const HostTable& h, int n, double v) {
    const double* s = h.buf.data();
    const int* bidx = reinterpret_cast<const int*>(h.buf.data() + h.off_bidx);
    double gf = (v - h.s0) * h.ibh;
    gf = gf > 0.0 ? gf : 0.0;
    const int g = gf < (double)(h.nb - 1) ? (int)gf : h.nb - 1;
    int lo = bidx[g > 0 ? g - 1 : 0];
    int hi = g + 2 <= h.nb ? bidx[g + 2] : h.T;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] < v) lo = mid + 1; else hi = mid;
    }
    lo = lo < n ? lo : n;
    lo = lo < 1 ? 1 : lo;
    lo = lo > n - 1 ? n - 1 : lo;
    return lo;
}

}  // namespace mpcqp_host

#endif  // MPCQP_HOST_TABLE_H
