// bed.cpp -- host-side BED / genome-file readers (the on-disk formats either
// side of the hot path; replaces ADAM sc.loadBed and the genome-file parse of
// cli/Complement.scala:43-44).  Pure C++, no device code.
//
// BED rules (ADAM's BED parser is 3rd-party and not vendored; parity of these
// corner cases is unpinned by any lime test):
//   - fields are tab-separated (whitespace if a line has no tab);
//   - empty lines and lines starting with '#', "track" or "browser" are skipped;
//   - columns: chrom, start, end [, name [, score [, strand]]]; start/end
//     are taken verbatim (0-based half-open);
//   - strand '+' -> 1, '-' -> 2, '?' -> 3, anything else (incl. '.') -> 0.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lime_amd.h"

namespace lime {
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
}  // namespace lime

struct lime_bed {
    std::vector<std::string> contig_names;
    std::vector<int32_t> contig;
    std::vector<int64_t> start, end;
    std::vector<int8_t> strand;
    std::vector<std::string> name;
};

namespace {

bool read_file(const char *path, std::string &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, k);
    fclose(f);
    return true;
}

void split(const char *b, const char *e, std::vector<std::pair<const char *, const char *>> &f) {
    f.clear();
    bool tab = memchr(b, '\t', (size_t)(e - b)) != nullptr;
    const char *p = b;
    if (tab) {
        while (true) {
            const char *q = (const char *)memchr(p, '\t', (size_t)(e - p));
            if (!q) {
                f.push_back({p, e});
                break;
            }
            f.push_back({p, q});
            p = q + 1;
        }
    } else {
        while (p < e) {
            while (p < e && (*p == ' ')) ++p;
            if (p >= e) break;
            const char *q = p;
            while (q < e && *q != ' ') ++q;
            f.push_back({p, q});
            p = q;
        }
    }
}

bool parse_i64(const char *b, const char *e, int64_t &v) {
    while (b < e && (*b == ' ')) ++b;
    while (e > b && (e[-1] == ' ')) --e;
    if (b >= e) return false;
    bool neg = false;
    if (*b == '-' || *b == '+') {
        neg = *b == '-';
        ++b;
    }
    if (b >= e) return false;
    int64_t x = 0;
    for (; b < e; ++b) {
        if (*b < '0' || *b > '9') return false;
        x = x * 10 + (*b - '0');
    }
    v = neg ? -x : x;
    return true;
}

bool starts_with(const char *b, const char *e, const char *p) {
    size_t n = strlen(p);
    return (size_t)(e - b) >= n && memcmp(b, p, n) == 0;
}

}  // namespace

extern "C" {

int lime_bed_read(const char *path, lime_bed **out) {
    if (!path || !out) return lime::fail(LIME_ERR_ARG, "bad bed arguments");
    std::string text;
    if (!read_file(path, text)) return lime::fail(LIME_ERR_IO, std::string("cannot read ") + path);
    lime_bed *bed = new lime_bed();
    std::unordered_map<std::string, int32_t> ids;
    std::vector<std::pair<const char *, const char *>> f;
    const char *p = text.data(), *end = text.data() + text.size();
    int64_t lineno = 0;
    while (p < end) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        const char *lb = p;
        p = nl ? nl + 1 : end;
        ++lineno;
        const char *ee = le;
        if (ee > lb && ee[-1] == '\r') --ee;
        if (ee == lb) continue;
        if (*lb == '#' || starts_with(lb, ee, "track") || starts_with(lb, ee, "browser")) continue;
        split(lb, ee, f);
        int64_t s, e;
        if (f.size() < 3 || !parse_i64(f[1].first, f[1].second, s) ||
            !parse_i64(f[2].first, f[2].second, e)) {
            delete bed;
            return lime::fail(LIME_ERR_IO, std::string(path) + ":" + std::to_string(lineno) +
                                               ": not a BED record");
        }
        std::string chrom(f[0].first, f[0].second);
        auto it = ids.find(chrom);
        int32_t id;
        if (it == ids.end()) {
            id = (int32_t)bed->contig_names.size();
            ids.emplace(chrom, id);
            bed->contig_names.push_back(chrom);
        } else {
            id = it->second;
        }
        bed->contig.push_back(id);
        bed->start.push_back(s);
        bed->end.push_back(e);
        bed->name.push_back(f.size() > 3 ? std::string(f[3].first, f[3].second) : std::string());
        int8_t st = 0;
        if (f.size() > 5 && f[5].second > f[5].first) {
            char c = *f[5].first;
            st = c == '+' ? 1 : c == '-' ? 2 : c == '?' ? 3 : 0;
        }
        bed->strand.push_back(st);
    }
    *out = bed;
    return LIME_OK;
}

int64_t lime_bed_rows(const lime_bed *b) { return b ? (int64_t)b->contig.size() : -1; }
int32_t lime_bed_contigs(const lime_bed *b) { return b ? (int32_t)b->contig_names.size() : -1; }
const char *lime_bed_contig_name(const lime_bed *b, int32_t i) {
    return (b && i >= 0 && i < (int32_t)b->contig_names.size()) ? b->contig_names[i].c_str()
                                                                 : nullptr;
}
const int32_t *lime_bed_contig_ids(const lime_bed *b) { return b ? b->contig.data() : nullptr; }
const int64_t *lime_bed_starts(const lime_bed *b) { return b ? b->start.data() : nullptr; }
const int64_t *lime_bed_ends(const lime_bed *b) { return b ? b->end.data() : nullptr; }
const int8_t *lime_bed_strands(const lime_bed *b) { return b ? b->strand.data() : nullptr; }
const char *lime_bed_name(const lime_bed *b, int64_t row) {
    return (b && row >= 0 && row < (int64_t)b->name.size()) ? b->name[row].c_str() : nullptr;
}
void lime_bed_free(lime_bed *b) { delete b; }

int lime_genome_read(const char *path, int32_t *n_out, char ***names_out, int64_t **lengths_out) {
    if (!path || !n_out || !names_out || !lengths_out)
        return lime::fail(LIME_ERR_ARG, "bad genome arguments");
    std::string text;
    if (!read_file(path, text)) return lime::fail(LIME_ERR_IO, std::string("cannot read ") + path);
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    std::vector<std::pair<const char *, const char *>> f;
    const char *p = text.data(), *end = text.data() + text.size();
    int64_t lineno = 0;
    while (p < end) {
        const char *nl = (const char *)memchr(p, '\n', (size_t)(end - p));
        const char *le = nl ? nl : end;
        const char *lb = p;
        p = nl ? nl + 1 : end;
        ++lineno;
        const char *ee = le;
        if (ee > lb && ee[-1] == '\r') --ee;
        if (ee == lb || *lb == '#') continue;
        split(lb, ee, f);
        int64_t len;
        if (f.size() < 2 || !parse_i64(f[1].first, f[1].second, len) || len < 0)
            return lime::fail(LIME_ERR_IO, std::string(path) + ":" + std::to_string(lineno) +
                                               ": expected name<TAB>length");
        names.emplace_back(f[0].first, f[0].second);
        lens.push_back(len);
    }
    int32_t n = (int32_t)names.size();
    char **nm = (char **)malloc(sizeof(char *) * (size_t)(n > 0 ? n : 1));
    int64_t *ln = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    for (int32_t i = 0; i < n; ++i) {
        nm[i] = strdup(names[i].c_str());
        ln[i] = lens[i];
    }
    *n_out = n;
    *names_out = nm;
    *lengths_out = ln;
    return LIME_OK;
}

void lime_genome_free(int32_t n, char **names, int64_t *lengths) {
    if (names)
        for (int32_t i = 0; i < n; ++i) free(names[i]);
    free(names);
    free(lengths);
}

}  // extern "C"
