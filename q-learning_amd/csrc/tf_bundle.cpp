// Reader of TensorFlow tensor bundles (a SavedModel's variables/variables.index + variables.data-*), the format
// the reference's models and checkpoints are stored in: saved/ql_model_*/variables (SavedModel export,
// create_ql_model_*.py model.save) and write_checkpoint (q_learning_model.rs:191-202, .py checkpoint.write).
//
// Format (restated from TF's tensor_bundle and LevelDB's table format; TF itself is not available here):
//   variables.index is an SSTable: ... data blocks ..., metaindex block, index block, 48-byte footer
//     footer = metaindex handle, index handle (varint64 offset + varint64 size each), zero padding to 40 bytes,
//              magic 0xdb4775248b80fb57 (little endian)
//     block  = entries {varint32 shared, varint32 non_shared, varint32 value_len, key suffix, value}, then
//              uint32 restart offsets and uint32 restart count; every block is followed by a 5-byte trailer
//              (compression type byte = 0, masked crc32c)
//     index block values are BlockHandles of the data blocks; data block keys are tensor names ("" = the
//     BundleHeaderProto) and values BundleEntryProto {1 dtype, 2 TensorShapeProto {2 dim {1 size}}, 3 shard_id,
//     4 offset, 5 size, 6 fixed32 masked crc32c of the tensor bytes}
//   variables.data-00000-of-00001 holds the raw little-endian tensor bytes at (offset, size).
// Host code only (no GPU calls): usable on a machine without a GPU.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "objects.h"
#include "qlx_internal.h"

namespace qlx {

namespace {

uint32_t crc32c_table[256];
bool crc_init = false;

uint32_t crc32c(const uint8_t* p, size_t n) {   // Castagnoli, reflected 0x82F63B78
  if (!crc_init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      crc32c_table[i] = c;
    }
    crc_init = true;
  }
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = crc32c_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }   // leveldb / tf crc32c::Mask

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64 && p < end; s += 7) {
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
  uint32_t fixed32() {
    if (end - p < 4) { ok = false; return 0; }
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  void skip(uint64_t n) {
    if ((uint64_t)(end - p) < n) { ok = false; p = end; return; }
    p += n;
  }
};

}  // namespace

struct BundleEntry {
  std::string name;
  int32_t dtype = 0;
  std::vector<int64_t> shape;
  int32_t shard = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;
  bool has_crc = false;
};

static bool parse_entry(const uint8_t* v, size_t n, BundleEntry& e) {   // BundleEntryProto
  Reader r{v, v + n};
  while (r.ok && r.p < r.end) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (wt == 0) {
      const uint64_t x = r.varint();
      if (field == 1) e.dtype = (int32_t)x;
      else if (field == 3) e.shard = (int32_t)x;
      else if (field == 4) e.offset = (int64_t)x;
      else if (field == 5) e.size = (int64_t)x;
    } else if (wt == 5) {
      const uint32_t x = r.fixed32();
      if (field == 6) { e.crc = x; e.has_crc = true; }
    } else if (wt == 2) {
      const uint64_t len = r.varint();
      if (field == 2) {   // TensorShapeProto: repeated Dim dim = 2 {int64 size = 1}
        Reader s{r.p, r.p + len};
        while (s.ok && s.p < s.end) {
          const uint64_t t2 = s.varint();
          if ((t2 >> 3) == 2 && (t2 & 7) == 2) {
            const uint64_t dl = s.varint();
            Reader d{s.p, s.p + dl};
            int64_t size = 0;
            while (d.ok && d.p < d.end) {
              const uint64_t t3 = d.varint();
              if ((t3 & 7) == 0) { const uint64_t x = d.varint(); if ((t3 >> 3) == 1) size = (int64_t)x; }
              else if ((t3 & 7) == 2) d.skip(d.varint());
              else { d.ok = false; }
            }
            e.shape.push_back(size);
            s.skip(dl);
          } else if ((t2 & 7) == 0) {
            s.varint();
          } else if ((t2 & 7) == 2) {
            s.skip(s.varint());
          } else {
            s.ok = false;
          }
        }
      }
      r.skip(len);
    } else if (wt == 1) {
      r.skip(8);
    } else {
      return false;
    }
  }
  return r.ok;
}

// entries of one SSTable block (keys prefix-compressed); values are handed to f(key, value ptr, len)
template <class F>
static void for_each_entry(const uint8_t* blk, size_t n, F f) {
  QLX_CHECK(n >= 4, QLX_E_IO, "tf bundle: short block");
  uint32_t restarts;
  std::memcpy(&restarts, blk + n - 4, 4);
  QLX_CHECK((size_t)restarts * 4 + 4 <= n, QLX_E_IO, "tf bundle: bad restart array");
  const uint8_t* end = blk + n - 4 - (size_t)restarts * 4;
  Reader r{blk, end};
  std::string key;
  while (r.ok && r.p < r.end) {
    const uint64_t shared = r.varint(), non_shared = r.varint(), vlen = r.varint();
    QLX_CHECK(r.ok && shared <= key.size() && (uint64_t)(r.end - r.p) >= non_shared + vlen, QLX_E_IO, "tf bundle: bad entry");
    key.resize(shared);
    key.append((const char*)r.p, non_shared);
    r.p += non_shared;
    f(key, r.p, (size_t)vlen);
    r.p += vlen;
  }
}

}  // namespace qlx

struct qlx_tf_bundle {
  std::string prefix;
  std::vector<qlx::BundleEntry> entries;
};

using namespace qlx;

static std::vector<uint8_t> read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  QLX_CHECK(f.good(), QLX_E_IO, "cannot open " + path);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

static const BundleEntry* find_entry(const qlx_tf_bundle* b, const std::string& name) {
  for (const auto& e : b->entries)
    if (e.name == name) return &e;
  return nullptr;
}

extern "C" {

int32_t qlx_tf_bundle_open(const char* prefix, qlx_tf_bundle** out) {
  return guard([&] {
    QLX_CHECK(prefix && out, QLX_E_INVALID, "null argument");
    auto* b = new qlx_tf_bundle;
    b->prefix = prefix;
    try {
      const std::vector<uint8_t> idx = read_file(b->prefix + ".index");
      QLX_CHECK(idx.size() >= 48, QLX_E_IO, "tf bundle: index shorter than a footer");
      const uint8_t* foot = idx.data() + idx.size() - 48;
      uint64_t magic;
      std::memcpy(&magic, foot + 40, 8);
      QLX_CHECK(magic == 0xdb4775248b80fb57ull, QLX_E_IO, "tf bundle: bad table magic");
      Reader fr{foot, foot + 40};
      fr.varint(); fr.varint();                       // metaindex handle (unused)
      const uint64_t io = fr.varint(), is = fr.varint();   // index handle
      QLX_CHECK(fr.ok && io + is + 5 <= idx.size(), QLX_E_IO, "tf bundle: bad index handle");
      auto check_block = [&](uint64_t off, uint64_t size) {
        QLX_CHECK(off + size + 5 <= idx.size(), QLX_E_IO, "tf bundle: block out of range");
        QLX_CHECK(idx[off + size] == 0, QLX_E_IO, "tf bundle: compressed blocks are not supported");
        uint32_t stored;
        std::memcpy(&stored, &idx[off + size + 1], 4);
        // the block crc covers the contents and the compression-type byte
        QLX_CHECK(crc_mask(crc32c(&idx[off], size + 1)) == stored, QLX_E_IO, "tf bundle: block checksum mismatch");
      };
      check_block(io, is);
      for_each_entry(&idx[io], (size_t)is, [&](const std::string&, const uint8_t* v, size_t n) {
        Reader h{v, v + n};
        const uint64_t off = h.varint(), size = h.varint();
        QLX_CHECK(h.ok, QLX_E_IO, "tf bundle: bad block handle");
        check_block(off, size);
        for_each_entry(&idx[off], (size_t)size, [&](const std::string& key, const uint8_t* ev, size_t en) {
          if (key.empty()) return;   // BundleHeaderProto
          BundleEntry e;
          e.name = key;
          QLX_CHECK(parse_entry(ev, en, e), QLX_E_IO, "tf bundle: bad entry proto for " + key);
          b->entries.push_back(e);
        });
      });
    } catch (...) {
      delete b;
      throw;
    }
    *out = b;
  });
}

int32_t qlx_tf_bundle_close(qlx_tf_bundle* b) {
  delete b;
  return QLX_OK;
}

int32_t qlx_tf_bundle_count(const qlx_tf_bundle* b) { return b ? (int32_t)b->entries.size() : -1; }

// entry i: name (NUL-terminated into name[cap]), TF DataType enum (1 float, 9 int64, ...), shape, byte size
int32_t qlx_tf_bundle_entry(const qlx_tf_bundle* b, int32_t i, char* name, size_t cap, int32_t* dtype, int64_t* dims,
                            int32_t* ndims, int64_t* nbytes) {
  return guard([&] {
    QLX_CHECK(b && i >= 0 && i < (int32_t)b->entries.size(), QLX_E_INVALID, "bad entry index");
    const BundleEntry& e = b->entries[i];
    if (name) {
      QLX_CHECK(e.name.size() < cap, QLX_E_INVALID, "name buffer too small");
      std::memcpy(name, e.name.c_str(), e.name.size() + 1);
    }
    if (dtype) *dtype = e.dtype;
    if (ndims) *ndims = (int32_t)e.shape.size();
    if (dims) for (size_t k = 0; k < e.shape.size() && k < 8; ++k) dims[k] = e.shape[k];
    if (nbytes) *nbytes = e.size;
  });
}

// raw little-endian bytes of tensor `name` from variables.data-<shard>-of-00001 (crc32c verified)
int32_t qlx_tf_bundle_read(const qlx_tf_bundle* b, const char* name, void* out, size_t cap) {
  return guard([&] {
    QLX_CHECK(b && name && out, QLX_E_INVALID, "null argument");
    const BundleEntry* e = find_entry(b, name);
    QLX_CHECK(e, QLX_E_INVALID, std::string("tf bundle: no tensor ") + name);
    QLX_CHECK((size_t)e->size <= cap, QLX_E_INVALID, "output buffer too small");
    char shard[64];
    std::snprintf(shard, sizeof shard, ".data-%05d-of-00001", e->shard);
    std::ifstream f(b->prefix + shard, std::ios::binary);
    QLX_CHECK(f.good(), QLX_E_IO, "cannot open " + b->prefix + shard);
    f.seekg(e->offset);
    f.read((char*)out, e->size);
    QLX_CHECK(f.gcount() == e->size, QLX_E_IO, "tf bundle: short data read");
    if (e->has_crc)
      QLX_CHECK(crc_mask(crc32c((const uint8_t*)out, (size_t)e->size)) == e->crc, QLX_E_IO,
                std::string("tf bundle: data checksum mismatch for ") + name);
  });
}

}  // extern "C"

namespace qlx {

void load_keras_bundle(const char* prefix, int n_layers, const int* var_sizes, std::vector<float>& w, std::vector<float>& m,
                       std::vector<float>& v, int64_t* iterations) {
  qlx_tf_bundle* b = nullptr;
  const int32_t st = qlx_tf_bundle_open(prefix, &b);
  QLX_CHECK(st == QLX_OK, st, qlx_last_error());
  try {
    size_t total = 0;
    for (int i = 0; i < 2 * n_layers; ++i) total += var_sizes[i];
    w.assign(total, 0.0f);
    m.assign(total, 0.0f);
    v.assign(total, 0.0f);
    size_t off = 0;
    for (int i = 0; i < 2 * n_layers; ++i) {
      const std::string base = "layer_with_weights-" + std::to_string(i / 2) + (i % 2 ? "/bias" : "/kernel");
      const std::string names[3] = {base + "/.ATTRIBUTES/VARIABLE_VALUE", base + "/.OPTIMIZER_SLOT/optimizer/m/.ATTRIBUTES/VARIABLE_VALUE",
                                    base + "/.OPTIMIZER_SLOT/optimizer/v/.ATTRIBUTES/VARIABLE_VALUE"};
      std::vector<float>* dst[3] = {&w, &m, &v};
      for (int k = 0; k < 3; ++k) {
        const BundleEntry* e = find_entry(b, names[k]);
        QLX_CHECK(e, QLX_E_INVALID, "tf bundle: missing " + names[k]);
        int64_t n = 1;
        for (int64_t d : e->shape) n *= d;
        QLX_CHECK(e->dtype == 1 && n == var_sizes[i] && e->size == n * 4, QLX_E_INVALID, "tf bundle: shape / dtype mismatch for " + names[k]);
        const int32_t r = qlx_tf_bundle_read(b, names[k].c_str(), dst[k]->data() + off, (size_t)n * 4);
        QLX_CHECK(r == QLX_OK, r, qlx_last_error());
      }
      off += var_sizes[i];
    }
    int64_t it = 0;
    const char* iter_name = "optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE";
    if (find_entry(b, iter_name)) {
      const int32_t r = qlx_tf_bundle_read(b, iter_name, &it, 8);
      QLX_CHECK(r == QLX_OK, r, qlx_last_error());
    }
    *iterations = it;
  } catch (...) {
    qlx_tf_bundle_close(b);
    throw;
  }
  qlx_tf_bundle_close(b);
}

}  // namespace qlx
