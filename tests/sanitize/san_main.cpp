// Host-side sanitizer driver (ASan + UBSan build, tests/sanitize/Makefile): runs the host
// parsers of libigx -- igx_filter_parse (filter.GetFilterFromString), igx_regex_compile_blob
// (the `~` rule's DFA compiler) and igx_sort_prepare (sort.Prepare) -- over a corpus of
// inputs, plus seeded random regex patterns and filter strings.  Test infrastructure only.
//
// corpus lines:  F <tab> filter string     (against the schema below)
//                R <tab> regex pattern
//                S <tab> sortBy entries separated by ','
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/igx.h"

namespace {

// the column set of pkg/columns/filter/filter_test.go's test struct, as the Python mirror
// describes it (tests/golden/filter_table.json)
const igx_schema_col kSchema[] = {
    {"string", IGX_KIND_BYTES, 16, 0, IGX_KIND_BYTES},  {"int", IGX_KIND_INT, 8, 0, IGX_KIND_INT},
    {"int8", IGX_KIND_INT, 1, 0, IGX_KIND_INT},         {"int16", IGX_KIND_INT, 2, 0, IGX_KIND_INT},
    {"int32", IGX_KIND_INT, 4, 0, IGX_KIND_INT},        {"int64", IGX_KIND_INT, 8, 0, IGX_KIND_INT},
    {"uint", IGX_KIND_UINT, 8, 0, IGX_KIND_UINT},       {"uint8", IGX_KIND_UINT, 1, 0, IGX_KIND_UINT},
    {"uint16", IGX_KIND_UINT, 2, 0, IGX_KIND_UINT},     {"uint32", IGX_KIND_UINT, 4, 0, IGX_KIND_UINT},
    {"uint64", IGX_KIND_UINT, 8, 0, IGX_KIND_UINT},     {"float32", IGX_KIND_FLOAT, 4, 0, IGX_KIND_FLOAT},
    {"float64", IGX_KIND_FLOAT, 8, 0, IGX_KIND_FLOAT},  {"bool", IGX_KIND_BOOL, 1, 0, IGX_KIND_BOOL},
    {"virt", IGX_KIND_BYTES, 16, IGX_COL_VIRTUAL, IGX_KIND_BYTES},
    {"ext", IGX_KIND_BYTES, 8, IGX_COL_EXTRACTOR, IGX_KIND_UINT},
};
constexpr uint32_t kN = sizeof kSchema / sizeof kSchema[0];

uint64_t rng_state = 0x5EED;
uint64_t next() {   // SplitMix64
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int run_filter(const std::string &f) {
    igx_pred p;
    char err[256];
    return igx_filter_parse(kSchema, kN, f.c_str(), &p, err, sizeof err);
}

int run_regex(const std::string &r) {
    size_t n = 0;
    char err[256];
    int rc = igx_regex_compile_blob(r.data(), r.size(), nullptr, 0, &n, err, sizeof err);
    if (rc == 0) {
        std::vector<uint8_t> buf(n);
        rc = igx_regex_compile_blob(r.data(), r.size(), buf.data(), buf.size(), &n, err, sizeof err);
    }
    return rc;
}

int run_sort(const std::string &s) {
    std::vector<std::string> parts;
    size_t a = 0;
    for (;;) {
        const size_t b = s.find(',', a);
        parts.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
    }
    std::vector<const char *> ptrs;
    for (auto &x : parts) ptrs.push_back(x.c_str());
    std::vector<igx_sortkey> out(parts.size() + 1);
    uint32_t n = 0, bad = 0;
    return igx_sort_prepare(kSchema, kN, ptrs.data(), (uint32_t)ptrs.size(), out.data(), &n, &bad);
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: san_main corpus.txt\n");
        return 2;
    }
    FILE *fp = std::fopen(argv[1], "rb");
    if (!fp) return 2;
    std::string line;
    long lines = 0, ok = 0;
    for (int ch; (ch = std::fgetc(fp)) != EOF || !line.empty();) {
        if (ch != '\n' && ch != EOF) {
            line.push_back((char)ch);
            continue;
        }
        if (line.size() >= 2 && line[1] == '\t') {
            const std::string arg = line.substr(2);
            int rc = 0;
            if (line[0] == 'F') rc = run_filter(arg);
            else if (line[0] == 'R') rc = run_regex(arg);
            else if (line[0] == 'S') rc = run_sort(arg);
            ++lines;
            ok += rc == 0;
        }
        line.clear();
        if (ch == EOF) break;
    }
    std::fclose(fp);
    // seeded random regex patterns and filter strings over the syntax's metacharacters
    static const char alpha[] = "ab(|)*+?{}[]^$\\.-:,0123456789dDwWsSbBpPQEzAimsxN{}é\xff~!<>=";
    long fuzz = 0;
    for (int i = 0; i < 15000; ++i) {
        std::string r;
        const int len = 1 + (int)(next() % 24);
        for (int k = 0; k < len; ++k) r.push_back(alpha[next() % (sizeof alpha - 1)]);
        run_regex(r);
        run_filter(std::string(kSchema[next() % kN].name) + ":" + r);
        ++fuzz;
    }
    std::printf("SAN_OK corpus=%ld parsed=%ld fuzz=%ld\n", lines, ok, fuzz);
    return 0;
}
