// pack.h — read-only access to assets_pack/<dir>.npz (tools/make_asset_packs.py), the asset
// store the GPU box receives: glTF JSON ("gltf:<rel>"), its buffers ("buf:<rel>:<i>") and every
// image decoded to 8-bit channels ("img:<rel>", H x W x C).  An npz is a zip of .npy files;
// entries are inflated with zlib.  Host side only, not part of the C ABI.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace rth {

struct NpyArray {
    std::string descr;            // numpy dtype string, e.g. "|u1", "<f4"
    std::vector<uint64_t> shape;
    std::vector<uint8_t> data;    // C order
};

class NpzFile {
  public:
    explicit NpzFile(const std::string& path);   // throws std::runtime_error
    bool has(const std::string& key) const { return entries_.count(key + ".npy") != 0; }
    NpyArray read(const std::string& key) const; // throws if absent or malformed

  private:
    struct Entry { uint64_t local_off, csize, usize; uint16_t method; };
    std::string path_;
    std::map<std::string, Entry> entries_;
};

// The pack store: assets addressed as in the scheme ("../../assets/<dir>/<rel>").
class PackStore {
  public:
    explicit PackStore(std::string root) : root_(std::move(root)) {}
    // (dir, rel) of a scheme asset path; throws on an empty path
    static void split(const std::string& path, std::string* dir, std::string* rel);
    const NpzFile* pack(const std::string& dir);  // nullptr when assets_pack/<dir>.npz is absent
    bool image(const std::string& path, NpyArray* out);  // false if the image is not in the pack

  private:
    std::string root_;
    std::map<std::string, std::unique_ptr<NpzFile>> open_;
};

}  // namespace rth
