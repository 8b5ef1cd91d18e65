// doc.h — the scheme document tree and its two readers (host side, not part of the C ABI).
//
// The reference reads schemes with serde_yaml (builder/mod.rs:63-67) and glTF JSON with the
// gltf crate.  Both land here as one tree:
//   * a YAML subset: block mappings and sequences by indentation, flow sequences [a, b],
//     plain / single- / double-quoted scalars, `#` comments, and serde's externally tagged
//     enums written as local tags (`- !Sphere`, `coloring: !Solid [..]`, a tag alone on a
//     line followed by its indented block);
//   * JSON (RFC 8259) — glTF documents and this repo's scene fixtures
//     (tests/golden/scenes/*.json, where a tag is an object with the single key "!Tag").
// A tagged value is a Tag node holding the tag name (without '!') and its value, whichever
// reader produced it.  Scalars keep their source text; numbers are parsed with strtod.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rth {

struct Node;
using NodeP = std::shared_ptr<Node>;

struct Node {
    enum Kind { Null, Scalar, String, Seq, Map, Tag } kind = Null;
    std::string text;                                  // Scalar / String text, Tag name
    std::vector<NodeP> seq;                            // Seq items; Tag: seq[0] is the value
    std::vector<std::pair<std::string, NodeP>> map;    // Map entries in document order

    const Node* get(const std::string& key) const;     // Map lookup (nullptr if absent)
    const Node* tagged() const { return kind == Tag && !seq.empty() ? seq[0].get() : nullptr; }
    bool is_true() const { return kind == Scalar && (text == "true" || text == "True" || text == "TRUE"); }
    double num() const;                                // strtod of a Scalar; throws otherwise
    const std::string& str() const;                    // Scalar or String text
};

// Both throw std::runtime_error with a line / offset on malformed input.
NodeP parse_yaml(const std::string& text);
NodeP parse_json(const std::string& text);

}  // namespace rth
