// Host-side GGUF v3 reader (ggml-free). Replaces the reference's use of
// gguf_init_from_file / gguf_find_key / gguf_get_tensor_* (magpie.cpp:73-121,
// 674-718; nano-codec.cpp:205-333). mmap-based; tensors are converted to f32 on
// demand (F32 / F16 / BF16 / Q8_0 / Q4_0; Q8_0 block = fp16 d + 32 x int8, Q4_0 block =
// fp16 d + 16 bytes of nibbles;
// scripts/convert_magpie_to_gguf.py:79-104).
#pragma once
#include <fcntl.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <map>
#include <string>
#include <vector>

namespace mp {

struct GgufTensor {
    std::string name;
    int type = 0;
    int n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    uint64_t offset = 0;
    int64_t nelements() const { return ne[0] * ne[1] * ne[2] * ne[3]; }
};

inline float half_to_float(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, exp = (h >> 10) & 0x1Fu, mant = h & 0x3FFu, x;
    if (exp == 0) {
        if (!mant) x = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(mant & 0x400u)) { mant <<= 1; exp--; }
            mant &= 0x3FFu;
            x = sign | (exp << 23) | (mant << 13);
        }
    } else if (exp == 31) x = sign | 0x7F800000u | (mant << 13);
    else x = sign | ((exp - 15 + 127) << 23) | (mant << 13);
    float f;
    memcpy(&f, &x, 4);
    return f;
}

class Gguf {
public:
    ~Gguf() { close(); }
    bool open(const std::string &path, std::string &err) {
        int fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) { err = "cannot open " + path; return false; }
        struct stat st;
        if (fstat(fd, &st) != 0) { ::close(fd); err = "cannot stat " + path; return false; }
        size_ = (size_t)st.st_size;
        void *m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
        ::close(fd);
        if (m == MAP_FAILED) { err = "mmap failed for " + path; return false; }
        map_ = (const uint8_t *)m;
        p_ = map_;
        end_ = map_ + size_;
        if (size_ < 24 || memcmp(map_, "GGUF", 4) != 0) { err = path + ": not a GGUF file"; return false; }
        p_ += 4;
        const uint32_t version = rd<uint32_t>();
        if (version != 3) { err = path + ": unsupported GGUF version " + std::to_string(version); return false; }
        const uint64_t nt = rd<uint64_t>(), nkv = rd<uint64_t>();
        uint64_t align = 32;
        for (uint64_t i = 0; i < nkv && ok_; ++i) {
            const std::string key = rd_str();
            const uint32_t type = rd<uint32_t>();
            read_value(key, type);
        }
        if (u32_.count("general.alignment")) align = u32_["general.alignment"];
        for (uint64_t i = 0; i < nt && ok_; ++i) {
            GgufTensor t;
            t.name = rd_str();
            t.n_dims = (int)rd<uint32_t>();
            if (t.n_dims < 1 || t.n_dims > 4) { ok_ = false; break; }
            for (int d = 0; d < t.n_dims; ++d) t.ne[d] = (int64_t)rd<uint64_t>();
            t.type = (int)rd<uint32_t>();
            t.offset = rd<uint64_t>();
            tensors_[t.name] = t;
        }
        if (!ok_) { err = path + ": truncated or malformed GGUF header"; return false; }
        const uint64_t pos = (uint64_t)(p_ - map_);
        data_off_ = (pos + align - 1) / align * align;
        for (auto &kv : tensors_) {
            const uint64_t nb = tensor_nbytes(kv.second);
            if (nb == 0 || data_off_ + kv.second.offset + nb > size_) {
                err = path + ": tensor " + kv.first + " has unsupported type or lies outside the file";
                return false;
            }
        }
        return true;
    }
    void close() {
        if (map_) munmap((void *)map_, size_);
        map_ = nullptr;
    }
    const GgufTensor *find(const std::string &name) const {
        auto it = tensors_.find(name);
        return it == tensors_.end() ? nullptr : &it->second;
    }
    int64_t get_u32(const std::string &key, int64_t def) const {
        auto it = u32_.find(key);
        return it == u32_.end() ? def : (int64_t)it->second;
    }
    bool get_str(const std::string &key, std::string &out) const {
        auto it = str_.find(key);
        if (it == str_.end()) return false;
        out = it->second;
        return true;
    }
    double get_f32(const std::string &key, double def) const {
        auto it = f32_.find(key);
        return it == f32_.end() ? def : it->second;
    }
    static uint64_t tensor_nbytes(const GgufTensor &t) {
        const int64_t n = t.nelements();
        switch (t.type) {
        case 0: return (uint64_t)n * 4;            // F32
        case 1: return (uint64_t)n * 2;            // F16
        case 30: return (uint64_t)n * 2;           // BF16
        case 8: return (uint64_t)(n / 32) * 34;    // Q8_0
        case 2: return (uint64_t)(n / 32) * 18;    // Q4_0
        default: return 0;
        }
    }
    // f32 copy of a tensor (dequantising), appended to `out`.
    bool to_f32(const GgufTensor &t, float *out) const {
        const uint8_t *src = map_ + data_off_ + t.offset;
        const int64_t n = t.nelements();
        switch (t.type) {
        case 0: memcpy(out, src, (size_t)n * 4); return true;
        case 1:
            for (int64_t i = 0; i < n; ++i) { uint16_t h; memcpy(&h, src + 2 * i, 2); out[i] = half_to_float(h); }
            return true;
        case 30:
            for (int64_t i = 0; i < n; ++i) {
                uint16_t h; memcpy(&h, src + 2 * i, 2);
                const uint32_t x = (uint32_t)h << 16; memcpy(&out[i], &x, 4);
            }
            return true;
        case 8:
            for (int64_t b = 0; b < n / 32; ++b) {
                const uint8_t *blk = src + b * 34;
                uint16_t h; memcpy(&h, blk, 2);
                const float d = half_to_float(h);
                for (int i = 0; i < 32; ++i) out[b * 32 + i] = (float)(int8_t)blk[2 + i] * d;
            }
            return true;
        case 2:  // Q4_0 (dequantize_row_q4_0): byte j holds q_j (low nibble) and q_{j+16}
            for (int64_t b = 0; b < n / 32; ++b) {
                const uint8_t *blk = src + b * 18;
                uint16_t h; memcpy(&h, blk, 2);
                const float d = half_to_float(h);
                for (int j = 0; j < 16; ++j) {
                    out[b * 32 + j] = (float)((int)(blk[2 + j] & 0x0F) - 8) * d;
                    out[b * 32 + j + 16] = (float)((int)(blk[2 + j] >> 4) - 8) * d;
                }
            }
            return true;
        }
        return false;
    }
    const std::map<std::string, GgufTensor> &tensors() const { return tensors_; }
    // the tensor's bytes as stored in the file (e.g. Q8_0 blocks)
    const uint8_t *data(const GgufTensor &t) const { return map_ + data_off_ + t.offset; }

private:
    template <class T> T rd() {
        T v{};
        if (p_ + sizeof(T) > end_) { ok_ = false; return v; }
        memcpy(&v, p_, sizeof(T));
        p_ += sizeof(T);
        return v;
    }
    std::string rd_str() {
        const uint64_t n = rd<uint64_t>();
        if (!ok_ || p_ + n > end_) { ok_ = false; return {}; }
        std::string s((const char *)p_, (size_t)n);
        p_ += n;
        return s;
    }
    void read_value(const std::string &key, uint32_t type) {
        static const int sz[13] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};
        if (type == 8) {
            std::string v = rd_str();
            if (!key.empty()) str_[key] = std::move(v);
            return;
        }
        if (type == 9) {
            const uint32_t et = rd<uint32_t>();
            const uint64_t n = rd<uint64_t>();
            for (uint64_t i = 0; i < n && ok_; ++i) read_value(std::string(), et);
            return;
        }
        if (type > 12) { ok_ = false; return; }
        if (p_ + sz[type] > end_) { ok_ = false; return; }
        const uint8_t *v = p_;
        p_ += sz[type];
        if (key.empty()) return;
        switch (type) {
        case 4: { uint32_t x; memcpy(&x, v, 4); u32_[key] = x; } break;
        case 5: { int32_t x; memcpy(&x, v, 4); u32_[key] = (uint64_t)(int64_t)x; } break;
        case 10: case 11: { uint64_t x; memcpy(&x, v, 8); u32_[key] = x; } break;
        case 6: { float x; memcpy(&x, v, 4); f32_[key] = x; } break;
        case 12: { double x; memcpy(&x, v, 8); f32_[key] = x; } break;
        default: break;
        }
    }
    const uint8_t *map_ = nullptr, *p_ = nullptr, *end_ = nullptr;
    size_t size_ = 0;
    uint64_t data_off_ = 0;
    bool ok_ = true;
    std::map<std::string, GgufTensor> tensors_;
    std::map<std::string, uint64_t> u32_;
    std::map<std::string, double> f32_;
    std::map<std::string, std::string> str_;
};

}  // namespace mp
