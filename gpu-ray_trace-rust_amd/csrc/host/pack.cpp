// pack.cpp — npz (zip of .npy) reader for the asset packs (pack.h).
#include "pack.h"

#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>

namespace rth {

namespace {

uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

std::vector<uint8_t> read_range(const std::string& path, uint64_t off, uint64_t n) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    f.seekg((std::streamoff)off);
    std::vector<uint8_t> b(n);
    f.read(reinterpret_cast<char*>(b.data()), (std::streamsize)n);
    if ((uint64_t)f.gcount() != n) throw std::runtime_error("short read in " + path);
    return b;
}

// Parses a .npy v1/v2/v3 header: {'descr': ..., 'fortran_order': False, 'shape': (..), }
void parse_npy(const std::vector<uint8_t>& raw, NpyArray* out) {
    if (raw.size() < 10 || std::memcmp(raw.data(), "\x93NUMPY", 6) != 0) throw std::runtime_error("not an .npy entry");
    const int major = raw[6];
    size_t hlen, hoff;
    if (major == 1) {
        hlen = rd16(&raw[8]);
        hoff = 10;
    } else {
        hlen = rd32(&raw[8]);
        hoff = 12;
    }
    if (hoff + hlen > raw.size()) throw std::runtime_error("truncated .npy header");
    const std::string h(reinterpret_cast<const char*>(&raw[hoff]), hlen);
    auto field = [&](const char* key) -> std::string {
        const size_t k = h.find(std::string("'") + key + "'");
        if (k == std::string::npos) throw std::runtime_error(std::string(".npy header lacks ") + key);
        size_t v = h.find(':', k) + 1;
        while (v < h.size() && h[v] == ' ') ++v;
        return h.substr(v);
    };
    std::string d = field("descr");
    if (d.empty() || d[0] != '\'') throw std::runtime_error("bad .npy descr");
    out->descr = d.substr(1, d.find('\'', 1) - 1);
    if (field("fortran_order").compare(0, 5, "False") != 0) throw std::runtime_error("fortran-order .npy");
    std::string s = field("shape");
    if (s.empty() || s[0] != '(') throw std::runtime_error("bad .npy shape");
    out->shape.clear();
    size_t p = 1;
    while (p < s.size() && s[p] != ')') {
        while (p < s.size() && (s[p] == ' ' || s[p] == ',')) ++p;
        if (p < s.size() && s[p] == ')') break;
        size_t e = p;
        while (e < s.size() && s[e] >= '0' && s[e] <= '9') ++e;
        if (e == p) throw std::runtime_error("bad .npy shape");
        out->shape.push_back(std::stoull(s.substr(p, e - p)));
        p = e;
    }
    out->data.assign(raw.begin() + (long)(hoff + hlen), raw.end());
}

}  // namespace

NpzFile::NpzFile(const std::string& path) : path_(path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot open " + path);
    const uint64_t size = (uint64_t)f.tellg();
    const uint64_t tail_n = size < 65557 ? size : 65557;  // EOCD + max comment
    std::vector<uint8_t> tail = read_range(path, size - tail_n, tail_n);
    long eocd = -1;
    for (long i = (long)tail_n - 22; i >= 0; --i)
        if (rd32(&tail[(size_t)i]) == 0x06054b50u) {
            eocd = i;
            break;
        }
    if (eocd < 0) throw std::runtime_error("not a zip file: " + path);
    uint64_t n = rd16(&tail[(size_t)eocd + 10]);
    uint64_t cd_size = rd32(&tail[(size_t)eocd + 12]);
    uint64_t cd_off = rd32(&tail[(size_t)eocd + 16]);
    // ZIP64 end-of-central-directory locator (just before the EOCD record)
    if (eocd >= 20 && rd32(&tail[(size_t)eocd - 20]) == 0x07064b50u) {
        const uint64_t z64 = rd64(&tail[(size_t)eocd - 12]);
        std::vector<uint8_t> r = read_range(path, z64, 56);
        if (rd32(r.data()) != 0x06064b50u) throw std::runtime_error("bad ZIP64 record: " + path);
        n = rd64(&r[32]);
        cd_size = rd64(&r[40]);
        cd_off = rd64(&r[48]);
    }
    std::vector<uint8_t> cd = read_range(path, cd_off, cd_size);
    size_t p = 0;
    for (uint64_t k = 0; k < n; ++k) {
        if (p + 46 > cd.size() || rd32(&cd[p]) != 0x02014b50u) throw std::runtime_error("bad central directory: " + path);
        Entry e{};
        e.method = rd16(&cd[p + 10]);
        e.csize = rd32(&cd[p + 20]);
        e.usize = rd32(&cd[p + 24]);
        const uint16_t nl = rd16(&cd[p + 28]), xl = rd16(&cd[p + 30]), cl = rd16(&cd[p + 32]);
        e.local_off = rd32(&cd[p + 42]);
        const std::string name(reinterpret_cast<const char*>(&cd[p + 46]), nl);
        // ZIP64 extended information: the 0xFFFFFFFF fields, in order usize, csize, offset
        size_t x = p + 46 + nl;
        const size_t xe = x + xl;
        while (x + 4 <= xe) {
            const uint16_t id = rd16(&cd[x]), len = rd16(&cd[x + 2]);
            if (id == 0x0001) {
                size_t q = x + 4;
                if (e.usize == 0xFFFFFFFFu) { e.usize = rd64(&cd[q]); q += 8; }
                if (e.csize == 0xFFFFFFFFu) { e.csize = rd64(&cd[q]); q += 8; }
                if (e.local_off == 0xFFFFFFFFu) { e.local_off = rd64(&cd[q]); q += 8; }
            }
            x += 4 + len;
        }
        entries_[name] = e;
        p += 46 + nl + xl + cl;
    }
}

NpyArray NpzFile::read(const std::string& key) const {
    auto it = entries_.find(key + ".npy");
    if (it == entries_.end()) throw std::runtime_error("no entry '" + key + "' in " + path_);
    const Entry& e = it->second;
    std::vector<uint8_t> lh = read_range(path_, e.local_off, 30);
    if (rd32(lh.data()) != 0x04034b50u) throw std::runtime_error("bad local header in " + path_);
    const uint64_t data_off = e.local_off + 30 + rd16(&lh[26]) + rd16(&lh[28]);
    std::vector<uint8_t> comp = read_range(path_, data_off, e.csize);
    std::vector<uint8_t> raw;
    if (e.method == 0) {
        raw = std::move(comp);
    } else if (e.method == 8) {
        raw.resize(e.usize);
        z_stream zs{};
        if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) throw std::runtime_error("inflateInit2 failed");
        zs.next_in = comp.data();
        zs.avail_in = (uInt)comp.size();
        zs.next_out = raw.data();
        zs.avail_out = (uInt)raw.size();
        const int r = inflate(&zs, Z_FINISH);
        inflateEnd(&zs);
        if (r != Z_STREAM_END || zs.total_out != raw.size()) throw std::runtime_error("inflate failed for " + key);
    } else {
        throw std::runtime_error("unsupported zip method in " + path_);
    }
    NpyArray a;
    parse_npy(raw, &a);
    return a;
}

void PackStore::split(const std::string& path, std::string* dir, std::string* rel) {
    std::vector<std::string> parts;
    size_t p = 0;
    while (p <= path.size()) {
        size_t e = path.find_first_of("/\\", p);
        if (e == std::string::npos) e = path.size();
        const std::string s = path.substr(p, e - p);
        if (!s.empty() && s != "." && s != "..") parts.push_back(s);
        p = e + 1;
    }
    if (!parts.empty() && parts[0] == "assets") parts.erase(parts.begin());
    if (parts.empty()) throw std::runtime_error("empty asset path");
    *dir = parts[0];
    rel->clear();
    for (size_t i = 1; i < parts.size(); ++i) *rel += (i > 1 ? "/" : "") + parts[i];
}

const NpzFile* PackStore::pack(const std::string& dir) {
    auto it = open_.find(dir);
    if (it != open_.end()) return it->second.get();
    const std::string p = root_ + "/" + dir + ".npz";
    std::unique_ptr<NpzFile> f;
    if (FILE* fp = std::fopen(p.c_str(), "rb")) {
        std::fclose(fp);
        f.reset(new NpzFile(p));
    }
    const NpzFile* r = f.get();
    open_[dir] = std::move(f);
    return r;
}

bool PackStore::image(const std::string& path, NpyArray* out) {
    std::string dir, rel;
    split(path, &dir, &rel);
    const NpzFile* pk = pack(dir);
    if (!pk || !pk->has("img:" + rel)) return false;
    *out = pk->read("img:" + rel);
    return true;
}

}  // namespace rth
