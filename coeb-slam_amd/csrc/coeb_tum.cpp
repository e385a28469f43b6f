// TUM RGB-D time-stamp lists and their association (host C++, no device code).
//
// Replaces the reference's associate.py (the ingest side of
// Tracking::GrabImageRGBD): read_file_list (associate.py:49-69) and associate (:71-102).
// Written from the published definition of the TUM association, not from that file:
//   * a list file is lines "stamp field field ..."; ',' and TAB separate like a space, a line
//     whose first byte is '#' is a comment, a line with fewer than two fields is ignored, and a
//     stamp that occurs twice keeps its last line;
//   * a pair (a, b) is a candidate when |a - (b + offset)| < max_difference, evaluated in double
//     exactly in that order;
//   * candidates are taken greedily by increasing (difference, a, b), each stamp at most once;
//   * the result is ordered by (a, b).
// Candidates come from a sorted copy of the second list and a window around a - offset, so the
// work is O((n + m) log m + k log k) for k candidates instead of the all-pairs O(n m).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <stdlib.h>
#include <unordered_map>
#include <vector>

#include "../../include/coeb_front.h"

namespace {

bool is_sep(char ch) { return ch == ' ' || ch == ',' || ch == '\t'; }
// what Python's str.strip() removes from an ASCII field besides the separators above
bool is_ws(char ch) { return ch == '\r' || ch == '\v' || ch == '\f' || ch == '\x1c' || ch == '\x1d' || ch == '\x1e' || ch == '\x1f'; }

struct Field { size_t b, e; };

// Fields of one line [b, e): split at separators, each trimmed, empty ones dropped.
void fields(const char* t, size_t b, size_t e, std::vector<Field>& out)
{
    out.clear();
    size_t i = b;
    while (i < e) {
        while (i < e && is_sep(t[i])) i++;
        size_t j = i;
        while (j < e && !is_sep(t[j])) j++;
        size_t fb = i, fe = j;
        while (fb < fe && is_ws(t[fb])) fb++;
        while (fe > fb && is_ws(t[fe - 1])) fe--;
        if (fe > fb) out.push_back({fb, fe});
        i = j;
    }
}

// The "C" numeric locale, created once: Python's float() does not depend on the locale, so a
// host that called setlocale(LC_NUMERIC, "de_DE") must still read '1305031102.175304'.
locale_t c_locale()
{
    static const locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    return loc;
}

// A decimal floating-point literal (optional sign, digits with at most one '.', optional
// exponent, or inf / infinity / nan), as a stamp field must be.  Hex forms are refused.
// Parsed in the "C" locale whatever the process locale is.
bool parse_stamp(const char* t, const Field& f, double* v)
{
    const size_t n = f.e - f.b;
    if (n == 0 || n > 127) return false;
    char buf[128];
    std::memcpy(buf, t + f.b, n);
    buf[n] = 0;
    const char* s = buf + ((buf[0] == '+' || buf[0] == '-') ? 1 : 0);
    if ((s[0] == '0' && (s[1] == 'x' || s[1] == 'X'))) return false;
    char* end = nullptr;
    const locale_t loc = c_locale();
    if (loc == (locale_t)0) return false;
    *v = strtod_l(buf, &end, loc);
    return end == buf + n;
}

}  // namespace

extern "C" int coeb_tum_read_list(const char* text, size_t len, double* stamps, int64_t* data_off, int32_t* data_len,
                                  int cap, int* n_out)
{
    if (!n_out || cap < 0 || (len > 0 && !text) || (cap > 0 && !stamps)) return COEB_EINVAL;
    *n_out = 0;
    std::vector<Field> fl;
    std::vector<double> st;
    std::vector<int64_t> off;
    std::vector<int32_t> dl;
    size_t b = 0;
    while (b <= len) {
        size_t e = b;
        while (e < len && text[e] != '\n') e++;
        if (e > b && text[b] != '#') {
            fields(text, b, e, fl);
            if (fl.size() > 1) {
                double v;
                if (!parse_stamp(text, fl[0], &v)) return COEB_EINVAL;   // float() of the first field raises
                st.push_back(v);
                off.push_back((int64_t)fl[1].b);
                dl.push_back((int32_t)(fl.back().e - fl[1].b));
            }
        }
        if (e >= len) break;
        b = e + 1;
    }
    // a repeated stamp keeps its last line, at the position of its first (Python dict insertion)
    std::unordered_map<double, size_t> first_at;
    std::vector<size_t> keep;
    for (size_t i = 0; i < st.size(); i++) {
        auto it = first_at.find(st[i]);
        if (std::isnan(st[i]) || it == first_at.end()) {
            if (!std::isnan(st[i])) first_at.emplace(st[i], keep.size());
            keep.push_back(i);
        } else {
            keep[it->second] = i;
        }
    }
    *n_out = (int)keep.size();
    if ((int)keep.size() > cap) return COEB_ERANGE;
    for (size_t k = 0; k < keep.size(); k++) {
        stamps[k] = st[keep[k]];
        if (data_off) data_off[k] = off[keep[k]];
        if (data_len) data_len[k] = dl[keep[k]];
    }
    return COEB_OK;
}

extern "C" int coeb_tum_associate(const double* first, int n_first, const double* second, int n_second, double offset,
                                  double max_difference, int32_t* first_idx, int32_t* second_idx, int cap, int* n_out)
{
    if (!n_out || n_first < 0 || n_second < 0 || cap < 0 || (n_first > 0 && !first) || (n_second > 0 && !second) ||
        (cap > 0 && (!first_idx || !second_idx)))
        return COEB_EINVAL;
    *n_out = 0;
    // each stamp value once (its last index), NaN stamps never match anything
    auto unique_last = [](const double* v, int n) {
        std::unordered_map<double, int> last;
        for (int i = 0; i < n; i++)
            if (!std::isnan(v[i])) last[v[i]] = i;
        std::vector<int> idx;
        idx.reserve(last.size());
        for (auto& kv : last) idx.push_back(kv.second);
        return idx;
    };
    const std::vector<int> A = unique_last(first, n_first);
    std::vector<int> B = unique_last(second, n_second);
    std::sort(B.begin(), B.end(), [&](int x, int y) { return second[x] < second[y]; });
    std::vector<double> bv(B.size());
    for (size_t j = 0; j < B.size(); j++) bv[j] = second[B[j]];

    struct Cand { double d, a, b; int ia, ib; };
    std::vector<Cand> cand;
    const bool windowed = std::isfinite(offset) && std::isfinite(max_difference);
    for (int ia : A) {
        const double a = first[ia];
        size_t j0 = 0, j1 = bv.size();
        if (windowed && std::isfinite(a)) {
            // b + offset within max_difference of a, widened by a few ulps of the operands so the
            // exact test below decides every boundary case
            const double slack = std::fabs(max_difference) +
                                 16.0 * DBL_EPSILON * (std::fabs(a) + std::fabs(offset) + std::fabs(max_difference));
            j0 = std::lower_bound(bv.begin(), bv.end(), a - offset - slack) - bv.begin();
            j1 = std::upper_bound(bv.begin(), bv.end(), a - offset + slack) - bv.begin();
        }
        for (size_t j = j0; j < j1; j++) {
            const double b = bv[j];
            const double d = std::fabs(a - (b + offset));
            if (d < max_difference) cand.push_back({d, a, b, ia, B[j]});
        }
    }
    std::sort(cand.begin(), cand.end(), [](const Cand& x, const Cand& y) {
        if (x.d != y.d) return x.d < y.d;
        if (x.a != y.a) return x.a < y.a;
        return x.b < y.b;
    });
    std::vector<char> used_a(n_first, 0), used_b(n_second, 0);
    std::vector<Cand> taken;
    for (const Cand& c : cand) {
        if (used_a[c.ia] || used_b[c.ib]) continue;
        used_a[c.ia] = used_b[c.ib] = 1;
        taken.push_back(c);
    }
    std::sort(taken.begin(), taken.end(), [](const Cand& x, const Cand& y) {
        if (x.a != y.a) return x.a < y.a;
        return x.b < y.b;
    });
    *n_out = (int)taken.size();
    if ((int)taken.size() > cap) return COEB_ERANGE;
    for (size_t k = 0; k < taken.size(); k++) {
        first_idx[k] = taken[k].ia;
        second_idx[k] = taken[k].ib;
    }
    return COEB_OK;
}
