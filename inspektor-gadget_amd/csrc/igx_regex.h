// igx_regex.h -- host-compiled regex DFA for the device filter scan (igx_regex.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

struct RegexDfa {
    static constexpr uint32_t MAXSTATES = 2048;
    static constexpr uint32_t MAXCLS = 4096;   // ASCII runes always fall in the first 128 classes
    uint32_t nstates = 0, ncls = 0, start = 0;
    std::vector<uint16_t> trans;      // nstates x ncls
    std::vector<uint8_t> flags;       // bit0 a match is complete (the absorbing accept state),
                                      // bit1 a match completes if the text ends here, bit2
                                      // (start state) the empty text matches
    std::vector<uint32_t> bounds;     // class k = runes [bounds[k], bounds[k+1]) (last: to U+10FFFF)
    uint8_t ascii[128] = {};          // class of each ASCII rune
};

// IGX_OK, IGX_EINVAL (syntax error: *why = the regexp/syntax message) or IGX_ENOTSUP
int igx_regex_compile(const char *pattern, size_t len, RegexDfa *dfa, std::string *why);

// device blob: header | ascii[128] | bounds[ncls] u32 | flags[nstates] u8 (padded to 4) |
// trans[nstates*ncls] u16
struct RegexBlobHeader {
    uint32_t nstates, ncls, start, bytes;
    uint32_t off_bounds, off_flags, off_trans, pad;
};
std::vector<uint8_t> igx_regex_blob(const RegexDfa &d);
