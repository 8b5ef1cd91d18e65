// doc.cpp — YAML-subset and JSON readers for the scheme / glTF document tree (doc.h).
#include "doc.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace rth {

const Node* Node::get(const std::string& key) const {
    if (kind != Map) return nullptr;
    for (const auto& kv : map)
        if (kv.first == key) return kv.second.get();
    return nullptr;
}

double Node::num() const {
    if (kind != Scalar) throw std::runtime_error("expected a number, got '" + text + "'");
    const char* b = text.c_str();
    char* e = nullptr;
    const double v = std::strtod(b, &e);
    if (e == b || *e != '\0') throw std::runtime_error("not a number: '" + text + "'");
    return v;
}

const std::string& Node::str() const {
    if (kind != Scalar && kind != String) throw std::runtime_error("expected a string");
    return text;
}

static NodeP make(Node::Kind k, std::string t = {}) {
    auto n = std::make_shared<Node>();
    n->kind = k;
    n->text = std::move(t);
    return n;
}

static std::string trim(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && std::isspace((unsigned char)s[b])) ++b;
    while (e > b && std::isspace((unsigned char)s[e - 1])) --e;
    return s.substr(b, e - b);
}

// ------------------------------------------------------------------------------- YAML subset
namespace {

struct Line {
    int indent;   // column of the first character
    int parent;   // a block value of this line must be indented more than this
    std::string s;
    int no;
};

[[noreturn]] void yerr(const Line& l, const std::string& what) {
    throw std::runtime_error("scheme YAML line " + std::to_string(l.no) + ": " + what);
}

std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (q) {
            if (c == q) q = 0;
        } else if (c == '"' || c == '\'') {
            q = c;
        } else if (c == '#' && (i == 0 || std::isspace((unsigned char)s[i - 1]))) {
            return s.substr(0, i);
        }
    }
    return s;
}

// Position of the mapping ':' (followed by space or end) outside quotes / brackets, or npos.
size_t key_colon(const std::string& s) {
    char q = 0;
    int depth = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        const char c = s[i];
        if (q) {
            if (c == q) q = 0;
            continue;
        }
        if (c == '"' || c == '\'') q = c;
        else if (c == '[' || c == '{') ++depth;
        else if (c == ']' || c == '}') --depth;
        else if (c == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ')) return i;
    }
    return std::string::npos;
}

std::string unquote(const std::string& s, bool* quoted) {
    *quoted = false;
    if (s.size() >= 2 && s.front() == '"' && s.back() == '"') {
        *quoted = true;
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); ++i) {
            if (s[i] == '\\' && i + 2 < s.size()) {
                const char n = s[++i];
                o += n == 'n' ? '\n' : (n == 't' ? '\t' : n);
            } else {
                o += s[i];
            }
        }
        return o;
    }
    if (s.size() >= 2 && s.front() == '\'' && s.back() == '\'') {
        *quoted = true;
        std::string o;
        for (size_t i = 1; i + 1 < s.size(); ++i) {
            o += s[i];
            if (s[i] == '\'' && i + 2 < s.size() && s[i + 1] == '\'') ++i;
        }
        return o;
    }
    return s;
}

NodeP scalar(const std::string& raw) {
    bool q;
    std::string t = unquote(trim(raw), &q);
    if (q) return make(Node::String, t);
    if (t.empty() || t == "~" || t == "null" || t == "Null" || t == "NULL") return make(Node::Null);
    return make(Node::Scalar, t);
}

class Flow {  // flow collections: [a, "b", [c]] and {k: v}
  public:
    Flow(const std::string& s, const Line& l) : s_(s), l_(l) {}
    NodeP parse() {
        NodeP n = value();
        ws();
        if (i_ != s_.size()) yerr(l_, "trailing text after flow collection");
        return n;
    }

  private:
    void ws() {
        while (i_ < s_.size() && std::isspace((unsigned char)s_[i_])) ++i_;
    }
    NodeP value() {
        ws();
        if (i_ >= s_.size()) yerr(l_, "unterminated flow collection");
        if (s_[i_] == '[') {
            ++i_;
            NodeP n = make(Node::Seq);
            ws();
            if (i_ < s_.size() && s_[i_] == ']') {
                ++i_;
                return n;
            }
            for (;;) {
                n->seq.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == ']') {
                    ++i_;
                    return n;
                }
                yerr(l_, "expected ',' or ']'");
            }
        }
        if (s_[i_] == '{') {
            ++i_;
            NodeP n = make(Node::Map);
            ws();
            if (i_ < s_.size() && s_[i_] == '}') {
                ++i_;
                return n;
            }
            for (;;) {
                NodeP k = atom(true);
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') yerr(l_, "expected ':' in flow mapping");
                ++i_;
                n->map.emplace_back(k->text, value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == '}') {
                    ++i_;
                    return n;
                }
                yerr(l_, "expected ',' or '}'");
            }
        }
        return atom(false);
    }
    NodeP atom(bool key) {
        ws();
        const size_t b = i_;
        if (i_ < s_.size() && (s_[i_] == '"' || s_[i_] == '\'')) {
            const char q = s_[i_++];
            while (i_ < s_.size() && !(s_[i_] == q && !(q == '"' && s_[i_ - 1] == '\\'))) ++i_;
            if (i_ >= s_.size()) yerr(l_, "unterminated quoted scalar");
            ++i_;
            return scalar(s_.substr(b, i_ - b));
        }
        while (i_ < s_.size() && s_[i_] != ',' && s_[i_] != ']' && s_[i_] != '}' && !(key && s_[i_] == ':')) ++i_;
        return scalar(s_.substr(b, i_ - b));
    }
    const std::string& s_;
    const Line& l_;
    size_t i_ = 0;
};

class Yaml {
  public:
    explicit Yaml(const std::string& text) {
        int no = 0;
        size_t p = 0;
        while (p <= text.size()) {
            size_t e = text.find('\n', p);
            if (e == std::string::npos) e = text.size();
            std::string raw = text.substr(p, e - p);
            ++no;
            p = e + 1;
            if (!raw.empty() && raw.back() == '\r') raw.pop_back();
            if (raw.find('\t') != std::string::npos && trim(raw).size() && raw.find_first_not_of(" \t") > raw.find('\t'))
                throw std::runtime_error("scheme YAML line " + std::to_string(no) + ": tab indentation");
            std::string s = strip_comment(raw);
            const std::string t = trim(s);
            if (t.empty() || t == "---" || t == "...") {
                if (e == text.size()) break;
                continue;
            }
            int ind = 0;
            while (ind < (int)s.size() && s[ind] == ' ') ++ind;
            lines_.push_back(Line{ind, ind, t, no});
            if (e == text.size()) break;
        }
    }
    NodeP parse() {
        if (lines_.empty()) return make(Node::Null);
        size_t i = 0;
        NodeP n = block(i);
        if (i != lines_.size()) yerr(lines_[i], "unexpected indentation");
        return n;
    }

  private:
    static bool is_dash(const std::string& s) { return s == "-" || (s.size() > 1 && s[0] == '-' && s[1] == ' '); }

    // The block starting at line i (its indentation is the block's).
    NodeP block(size_t& i) {
        const Line& l = lines_[i];
        if (is_dash(l.s)) return seq(i);
        if (l.s[0] == '!') return tag_line(i);
        if (key_colon(l.s) != std::string::npos && l.s[0] != '[' && l.s[0] != '{') return map(i);
        NodeP n = inline_value(l.s, l);
        ++i;
        return n;
    }

    // A block value following line `owner` (more indented than owner.parent), if any.
    NodeP child(size_t& i, const Line& owner, bool allow_seq_same_indent) {
        if (i < lines_.size()) {
            const Line& nx = lines_[i];
            if (nx.indent > owner.parent) return block(i);
            if (allow_seq_same_indent && nx.indent == owner.indent && is_dash(nx.s)) return block(i);
        }
        return make(Node::Null);
    }

    NodeP tag_line(size_t& i) {
        const Line l = lines_[i];
        size_t e = 1;
        while (e < l.s.size() && !std::isspace((unsigned char)l.s[e])) ++e;
        NodeP t = make(Node::Tag, l.s.substr(1, e - 1));
        const std::string rest = trim(l.s.substr(e));
        ++i;
        if (rest.empty()) t->seq.push_back(child(i, l, false));
        else t->seq.push_back(inline_value(rest, l));
        return t;
    }

    NodeP map(size_t& i) {
        const int ind = lines_[i].indent;
        NodeP m = make(Node::Map);
        while (i < lines_.size() && lines_[i].indent == ind && !is_dash(lines_[i].s)) {
            const Line l = lines_[i];
            const size_t c = key_colon(l.s);
            if (c == std::string::npos) yerr(l, "expected 'key: value'");
            bool q;
            const std::string key = unquote(trim(l.s.substr(0, c)), &q);
            const std::string rest = trim(l.s.substr(c + 1));
            ++i;
            NodeP v;
            if (rest.empty()) {
                Line owner = l;
                owner.parent = l.indent;
                v = child(i, owner, true);
            } else if (rest[0] == '!') {
                size_t e = 1;
                while (e < rest.size() && !std::isspace((unsigned char)rest[e])) ++e;
                v = make(Node::Tag, rest.substr(1, e - 1));
                const std::string r2 = trim(rest.substr(e));
                if (r2.empty()) {
                    Line owner = l;
                    owner.parent = l.indent;
                    v->seq.push_back(child(i, owner, false));
                } else {
                    v->seq.push_back(inline_value(r2, l));
                }
            } else {
                v = inline_value(rest, l);
            }
            m->map.emplace_back(key, v);
        }
        return m;
    }

    NodeP seq(size_t& i) {
        const int ind = lines_[i].indent;
        NodeP s = make(Node::Seq);
        while (i < lines_.size() && lines_[i].indent == ind && is_dash(lines_[i].s)) {
            Line& l = lines_[i];
            size_t b = 1;
            while (b < l.s.size() && l.s[b] == ' ') ++b;
            if (b >= l.s.size()) {  // "-" alone: the item is the following block
                const Line owner = l;
                ++i;
                s->seq.push_back(child(i, owner, false));
                continue;
            }
            // "- rest": rest is a virtual line at its own column; its block values must still be
            // indented more than the dash
            l.parent = ind;
            l.indent = ind + (int)b;
            l.s = l.s.substr(b);
            s->seq.push_back(block(i));
        }
        return s;
    }

    NodeP inline_value(const std::string& rest, const Line& l) {
        if (rest[0] == '[' || rest[0] == '{') return Flow(rest, l).parse();
        if (rest[0] == '!') {
            size_t e = 1;
            while (e < rest.size() && !std::isspace((unsigned char)rest[e])) ++e;
            NodeP t = make(Node::Tag, rest.substr(1, e - 1));
            const std::string r2 = trim(rest.substr(e));
            t->seq.push_back(r2.empty() ? make(Node::Null) : inline_value(r2, l));
            return t;
        }
        return scalar(rest);
    }

    std::vector<Line> lines_;
};

}  // namespace

NodeP parse_yaml(const std::string& text) { return Yaml(text).parse(); }

// ------------------------------------------------------------------------------------ JSON
namespace {

class Json {
  public:
    explicit Json(const std::string& s) : s_(s) {}
    NodeP parse() {
        NodeP n = value();
        ws();
        if (i_ != s_.size()) err("trailing characters");
        return n;
    }

  private:
    [[noreturn]] void err(const std::string& what) {
        throw std::runtime_error("JSON offset " + std::to_string(i_) + ": " + what);
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
    }
    bool lit(const char* w) {
        size_t k = 0;
        while (w[k]) {
            if (i_ + k >= s_.size() || s_[i_ + k] != w[k]) return false;
            ++k;
        }
        i_ += k;
        return true;
    }
    static void utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) {
            o += (char)cp;
        } else if (cp < 0x800) {
            o += (char)(0xC0 | (cp >> 6));
            o += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18));
            o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        }
    }
    uint32_t hex4() {
        if (i_ + 4 > s_.size()) err("bad \\u escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = s_[i_++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else err("bad \\u escape");
        }
        return v;
    }
    std::string string() {
        ++i_;  // opening quote
        std::string o;
        for (;;) {
            if (i_ >= s_.size()) err("unterminated string");
            const char c = s_[i_++];
            if (c == '"') return o;
            if (c != '\\') {
                o += c;
                continue;
            }
            if (i_ >= s_.size()) err("unterminated escape");
            const char e = s_[i_++];
            switch (e) {
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case '/': o += '/'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 1 < s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        i_ += 2;
                        const uint32_t lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(o, cp);
                    break;
                }
                default: err("bad escape");
            }
        }
    }
    NodeP value() {
        ws();
        if (i_ >= s_.size()) err("unexpected end");
        const char c = s_[i_];
        if (c == '{') {
            ++i_;
            NodeP m = make(Node::Map);
            ws();
            if (i_ < s_.size() && s_[i_] == '}') {
                ++i_;
                return m;
            }
            for (;;) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') err("expected a key");
                std::string k = string();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') err("expected ':'");
                ++i_;
                m->map.emplace_back(std::move(k), value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == '}') {
                    ++i_;
                    break;
                }
                err("expected ',' or '}'");
            }
            // {"!Tag": value} is a tagged value (the JSON form of a YAML local tag)
            if (m->map.size() == 1 && !m->map[0].first.empty() && m->map[0].first[0] == '!') {
                NodeP t = make(Node::Tag, m->map[0].first.substr(1));
                t->seq.push_back(m->map[0].second);
                return t;
            }
            return m;
        }
        if (c == '[') {
            ++i_;
            NodeP a = make(Node::Seq);
            ws();
            if (i_ < s_.size() && s_[i_] == ']') {
                ++i_;
                return a;
            }
            for (;;) {
                a->seq.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (i_ < s_.size() && s_[i_] == ']') {
                    ++i_;
                    return a;
                }
                err("expected ',' or ']'");
            }
        }
        if (c == '"') return make(Node::String, string());
        if (lit("true")) return make(Node::Scalar, "true");
        if (lit("false")) return make(Node::Scalar, "false");
        if (lit("null")) return make(Node::Null);
        const size_t b = i_;
        while (i_ < s_.size() && (std::isdigit((unsigned char)s_[i_]) || s_[i_] == '-' || s_[i_] == '+' ||
                                  s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E'))
            ++i_;
        if (b == i_) err("unexpected character");
        return make(Node::Scalar, s_.substr(b, i_ - b));
    }
    const std::string& s_;
    size_t i_ = 0;
};

}  // namespace

NodeP parse_json(const std::string& text) { return Json(text).parse(); }

}  // namespace rth

// ------------------------------------------------------------- test hook: the tree as JSON
namespace {
void dump(const rth::Node* n, std::string& o) {
    auto qs = [&](const std::string& s) {
        o += '"';
        for (char c : s) {
            if (c == '"' || c == '\\') o += '\\';
            if (c == '\n') { o += "\\n"; continue; }
            o += c;
        }
        o += '"';
    };
    switch (n->kind) {
        case rth::Node::Null: o += "null"; break;
        case rth::Node::Scalar:
        case rth::Node::String: qs(n->text); break;
        case rth::Node::Seq:
            o += '[';
            for (size_t i = 0; i < n->seq.size(); ++i) {
                if (i) o += ',';
                dump(n->seq[i].get(), o);
            }
            o += ']';
            break;
        case rth::Node::Map:
            o += '{';
            for (size_t i = 0; i < n->map.size(); ++i) {
                if (i) o += ',';
                qs(n->map[i].first);
                o += ':';
                dump(n->map[i].second.get(), o);
            }
            o += '}';
            break;
        case rth::Node::Tag:
            o += '{';
            qs("!" + n->text);
            o += ':';
            if (n->tagged()) dump(n->tagged(), o);
            else o += "null";
            o += '}';
            break;
    }
}
}  // namespace

// Not part of the ABI: the parsed document as JSON (scalars as strings), for tests.  Returns
// the length needed (writing at most cap bytes), or -1 on a parse error.
extern "C" long long rtx_doc_to_json(const char* text, unsigned long long len, unsigned format, char* out,
                                     unsigned long long cap) {
    try {
        const std::string src(text, (size_t)len);
        const rth::NodeP root = format == 0 ? rth::parse_yaml(src) : rth::parse_json(src);
        std::string o;
        dump(root.get(), o);
        if (out && cap) {
            const size_t n = o.size() < cap ? o.size() : (size_t)cap;
            for (size_t i = 0; i < n; ++i) out[i] = o[i];
        }
        return (long long)o.size();
    } catch (const std::exception&) {
        return -1;
    }
}
