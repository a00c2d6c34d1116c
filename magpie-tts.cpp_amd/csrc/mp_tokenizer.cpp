// Text front end of the reference (magpie.cpp:124-495): number/currency/percent/
// ordinal/year normalisation, ASCII lower-casing, punctuation split, IPA
// pronunciation-dictionary lookup with greedy longest-token (<= 4 bytes) matching,
// upper-case letter fallback for out-of-dictionary words, space tokens between
// words, BOS/EOS. Host C++ (string work, no device involvement); vocabulary and
// dictionary come from the GGUF strings magpie.tokenizer.vocab / .dict.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/magpie.h"
#include "mp_gguf.hpp"

namespace {

const char *kOnes[20] = {"zero",    "one",     "two",       "three",    "four",     "five",    "six",
                         "seven",   "eight",   "nine",      "ten",      "eleven",   "twelve",  "thirteen",
                         "fourteen", "fifteen", "sixteen",  "seventeen", "eighteen", "nineteen"};
const char *kTens[10] = {"", "", "twenty", "thirty", "forty", "fifty", "sixty", "seventy", "eighty", "ninety"};

// number_to_words (magpie.cpp:153-207)
std::string cardinal(int64_t n, bool with_and = true) {
    if (n < 0) return "minus " + cardinal(-n, with_and);
    if (n < 20) return kOnes[n];
    if (n < 100) return n % 10 ? std::string(kTens[n / 10]) + " " + kOnes[n % 10] : std::string(kTens[n / 10]);
    if (n < 1000) {
        std::string w = std::string(kOnes[n / 100]) + " hundred";
        if (n % 100) w += (with_and ? " and " : " ") + cardinal(n % 100, with_and);
        return w;
    }
    struct Scale { int64_t unit; const char *name; };
    // thousands cover 1,000..999,999 (the reference's 10,000+ branch is the same rule)
    static const Scale scales[3] = {{1000000000LL, " billion"}, {1000000LL, " million"}, {1000LL, " thousand"}};
    if (n >= 1000000000000LL) return std::to_string(n);
    for (const Scale &sc : scales) {
        if (n < sc.unit) continue;
        std::string w = cardinal(n / sc.unit, with_and) + sc.name;
        if (n % sc.unit) w += " " + cardinal(n % sc.unit, with_and);
        return w;
    }
    return std::to_string(n);
}

// year_to_words (210-227): 1900 -> "nineteen hundred", 2024 -> "twenty twenty four"
std::string year_words(int64_t n) {
    if (n < 1000 || n > 9999) return cardinal(n);
    const int64_t hi = n / 100, lo = n % 100;
    if (lo == 0) return cardinal(hi) + " hundred";
    if (lo < 10) return cardinal(n);
    return cardinal(hi) + " " + cardinal(lo);
}

// ordinal_to_words (230-262), including its compound rule: the last word of the
// cardinal is replaced by first/second/third when the last digit is 1/2/3
std::string ordinal(int64_t n) {
    static const char *special[13] = {"",      "first",  "second", "third",  "fourth", "fifth",   "sixth",
                                      "seventh", "eighth", "ninth",  "tenth",  "eleventh", "twelfth"};
    if (n >= 1 && n <= 12) return special[n];
    const std::string c = cardinal(n);
    if (n >= 13 && n <= 19) return c + "th";
    if (n >= 20 && n < 100 && n % 10 == 0) return c.back() == 'y' ? c.substr(0, c.size() - 1) + "ieth" : c + "th";
    const int last = (int)(n % 10);
    if (last >= 1 && last <= 3) {
        static const char *tail[4] = {"", "first", "second", "third"};
        const size_t sp = c.rfind(' ');
        return (sp == std::string::npos ? std::string() : c.substr(0, sp + 1)) + tail[last];
    }
    return c + "th";
}

bool is_digit(char c) { return c >= '0' && c <= '9'; }
char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c - 'A' + 'a') : c; }

// normalize_text (265-351)
std::string normalise(const std::string &t) {
    std::string out;
    out.reserve(t.size() * 2);
    size_t i = 0;
    auto digits = [&](int &count) {
        int64_t v = 0;
        count = 0;
        while (i < t.size() && is_digit(t[i])) {
            v = (int64_t)((uint64_t)v * 10u + (uint64_t)(t[i] - '0'));  // wraps like the reference's int64 on overlong runs
            ++count;
            ++i;
        }
        return v;
    };
    while (i < t.size()) {
        if (t[i] == '$' && i + 1 < t.size() && is_digit(t[i + 1])) {  // $50 -> "fifty dollars"
            ++i;
            int nd;
            const int64_t v = digits(nd);
            out += cardinal(v) + (v == 1 ? " dollar" : " dollars");
            continue;
        }
        const bool neg = t[i] == '-' && i + 1 < t.size() && is_digit(t[i + 1]);
        if (neg || is_digit(t[i])) {
            if (neg) ++i;
            int nd;
            const int64_t v = digits(nd);
            if (i < t.size() && t[i] == '%') {  // 50% -> "fifty percent"
                ++i;
                out += (neg ? "minus " : "") + cardinal(v) + " percent";
                continue;
            }
            bool ord = false;
            if (i + 1 < t.size()) {
                const char a = lower(t[i]), b = lower(t[i + 1]);
                ord = (a == 's' && b == 't') || (a == 'n' && b == 'd') || (a == 'r' && b == 'd') || (a == 't' && b == 'h');
                if (ord) i += 2;
            }
            std::string w = ord ? ordinal(v) : (nd == 4 && v >= 1000 && v <= 2099) ? year_words(v) : cardinal(v);
            if (neg && v != 0) w = "minus " + w;
            out += w;
            continue;
        }
        out += t[i++];
    }
    return out;
}

std::vector<std::string> split_on(const std::string &s, char sep) {
    std::vector<std::string> parts;
    size_t a = 0;
    for (size_t b; (b = s.find(sep, a)) != std::string::npos; a = b + 1) parts.push_back(s.substr(a, b - a));
    parts.push_back(s.substr(a));
    return parts;
}

}  // namespace

// the opaque GGUF handle of magpie.h (ggml-free: mp::Gguf, a read-only mapping)
struct gguf_context {
    mp::Gguf g;
};

struct gguf_context *magpie_gguf_open(const char *gguf_path) {
    if (!gguf_path) return nullptr;
    gguf_context *c = new gguf_context();
    std::string err;
    if (!c->g.open(gguf_path, err)) {
        fprintf(stderr, "magpie_gguf_open: %s\n", err.c_str());
        delete c;
        return nullptr;
    }
    return c;
}

void magpie_gguf_close(struct gguf_context *gguf_ctx) { delete gguf_ctx; }

// magpie_tokenizer_init (magpie.cpp:353-398): false when the GGUF carries no tokenizer
bool magpie_tokenizer_init(magpie_tokenizer *tok, struct gguf_context *gguf_ctx) {
    if (!tok || !gguf_ctx) return false;
    mp::Gguf &g = gguf_ctx->g;
    std::string vocab, dict;
    if (!g.get_str("magpie.tokenizer.vocab", vocab)) return false;
    tok->vocab = split_on(vocab, '\n');
    tok->token_to_id.clear();
    for (size_t i = 0; i < tok->vocab.size(); ++i) tok->token_to_id[tok->vocab[i]] = (int32_t)i;
    tok->dict.clear();
    if (g.get_str("magpie.tokenizer.dict", dict))
        for (const std::string &line : split_on(dict, '\n')) {
            const size_t tab = line.find('\t');
            if (tab != std::string::npos) tok->dict[line.substr(0, tab)] = line.substr(tab + 1);
        }
    tok->pad_id = (int32_t)g.get_u32("magpie.tokenizer.pad", 94);
    tok->oov_id = (int32_t)g.get_u32("magpie.tokenizer.oov", 95);
    tok->space_id = (int32_t)g.get_u32("magpie.tokenizer.space", 93);
    tok->bos_id = (int32_t)g.get_u32("magpie.text_bos_id", 2378);
    tok->eos_id = (int32_t)g.get_u32("magpie.text_eos_id", 2379);
    tok->loaded = true;
    return true;
}

bool magpie_tokenizer_load(magpie_tokenizer *tok, const char *gguf_path) {
    if (!tok || !gguf_path) return false;
    gguf_context *c = magpie_gguf_open(gguf_path);
    if (!c) return false;
    const bool ok = magpie_tokenizer_init(tok, c);
    magpie_gguf_close(c);
    return ok;
}

// magpie_tokenize (magpie.cpp:400-492)
std::vector<int32_t> magpie_tokenize(const magpie_tokenizer *tok, const std::string &text) {
    std::vector<int32_t> ids;
    if (!tok || !tok->loaded) return ids;
    ids.push_back(tok->bos_id);
    std::string norm = normalise(text), spaced;
    for (char &c : norm) c = lower(c);
    for (char c : norm) {
        if (strchr(",.!?:;", c) && c) {
            spaced += ' ';
            spaced += c;
            spaced += ' ';
        } else {
            spaced += c;
        }
    }
    auto id_of = [&](const std::string &s, int32_t &id) {
        auto it = tok->token_to_id.find(s);
        if (it == tok->token_to_id.end()) return false;
        id = it->second;
        return true;
    };
    for (const std::string &w : split_on(spaced, ' ')) {
        if (w.empty()) continue;
        int32_t id;
        if (w.size() == 1 && id_of(w, id)) {  // punctuation / single-char token: no space after it
            ids.push_back(id);
            continue;
        }
        auto d = tok->dict.find(w);
        if (d != tok->dict.end()) {
            const std::string &p = d->second;
            for (size_t i = 0; i < p.size();) {
                size_t n = std::min<size_t>(4, p.size() - i);
                for (; n > 0; --n)
                    if (id_of(p.substr(i, n), id)) break;
                if (n) { ids.push_back(id); i += n; }
                else ++i;  // byte with no token: skipped
            }
        } else {
            for (char c : w) {  // out-of-dictionary: upper-case letter tokens
                const char u = (c >= 'a' && c <= 'z') ? (char)(c - 'a' + 'A') : c;
                if (id_of(std::string(1, u), id)) ids.push_back(id);
            }
        }
        if (tok->space_id >= 0) ids.push_back(tok->space_id);
    }
    if (!ids.empty() && ids.back() == tok->space_id) ids.pop_back();
    ids.push_back(tok->eos_id);
    return ids;
}

// ---- C-ABI (magpie_hip.h)
struct mp_tokenizer { magpie_tokenizer t; };

extern "C" int mp_tokenizer_load(const char *gguf_path, mp_tokenizer **out) {
    if (!gguf_path || !out) return MP_ERR_ARG;
    mp_tokenizer *tk = new mp_tokenizer();
    if (!magpie_tokenizer_load(&tk->t, gguf_path)) {
        delete tk;
        return MP_ERR_FORMAT;
    }
    *out = tk;
    return MP_OK;
}

extern "C" int mp_tokenize(mp_tokenizer *tk, const char *text, int32_t *out, int cap) {
    if (!tk || !text || cap < 0 || (cap > 0 && !out)) return MP_ERR_ARG;
    const std::vector<int32_t> ids = magpie_tokenize(&tk->t, text);
    for (int i = 0; i < (int)ids.size() && i < cap; ++i) out[i] = ids[i];
    return (int)ids.size();
}

extern "C" void mp_tokenizer_free(mp_tokenizer *tk) { delete tk; }

// magpie_split_sentences (magpie.cpp:4439-4480): a sentence ends after . ! ?
// followed by whitespace (space, newline, tab) or the end of the text; leading
// whitespace of each piece is trimmed; a non-blank remainder is the last piece.
extern "C" int mp_split_sentences(const char *text, int32_t *offsets, int32_t *lengths, int cap) {
    if (!text || cap < 0) return MP_ERR_ARG;
    int count = 0;
    auto emit = [&](size_t a, size_t b) {  // piece [a, b): trim leading blanks
        while (a < b && strchr(" \t\n\r", text[a])) ++a;
        if (a == b) return;
        if (count < cap) {
            if (offsets) offsets[count] = (int32_t)a;
            if (lengths) lengths[count] = (int32_t)(b - a);
        }
        ++count;
    };
    size_t start = 0, i = 0;
    for (; text[i]; ++i) {
        const char c = text[i], nx = text[i + 1];
        if ((c == '.' || c == '!' || c == '?') && (nx == 0 || nx == ' ' || nx == '\n' || nx == '\t')) {
            emit(start, i + 1);
            start = i + 1;
        }
    }
    emit(start, i);
    return count;
}
