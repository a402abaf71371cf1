// TensorFlow TensorBundle checkpoint format, native writer + reader (SURVEY.md
// F21/N12; reference: RunConfig(model_dir, save_checkpoints_steps) at
// mnist_keras_distributed.py:245,248 makes TF write these files).
//
//   <prefix>.index                 LevelDB-format SSTable (no compression):
//                                  ""  -> BundleHeaderProto{num_shards=1, LITTLE, version{producer=1}}
//                                  key -> BundleEntryProto{dtype, shape, shard_id=0, offset, size, crc32c}
//   <prefix>.data-00000-of-00001   raw little-endian tensor bytes, concatenated
//
// SSTable details implemented here: data blocks with prefix-compressed keys and a
// restart point every 16 entries, 5-byte block trailer (type byte + masked
// crc32c over contents+type), index block (restart interval 1) of BlockHandles,
// empty metaindex block, 48-byte footer ending in magic 0xdb4775248b80fb57.
// Protobuf messages are hand-encoded in wire format.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#define TDE_API extern "C" __attribute__((visibility("default")))

namespace tde_host {
uint32_t crc32c(const void* data, size_t n);
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
uint32_t crc32c_mask(uint32_t crc);
uint32_t crc32c_unmask(uint32_t m);
}  // namespace tde_host

namespace {

using tde_host::crc32c;
using tde_host::crc32c_extend;
using tde_host::crc32c_mask;
using tde_host::crc32c_unmask;

constexpr uint64_t kMagic = 0xdb4775248b80fb57ull;
constexpr size_t kBlockSize = 262144;
constexpr int kRestartInterval = 16;

// ------------------------------------------------------------------ encoding helpers
void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)(v | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}
void put_fixed32(std::string* s, uint32_t v) { s->append((const char*)&v, 4); }
void put_fixed64(std::string* s, uint64_t v) { s->append((const char*)&v, 8); }

bool get_varint(const char*& p, const char* end, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint8_t b = (uint8_t)*p++;
    r |= (uint64_t)(b & 0x7F) << shift;
    if (!(b & 0x80)) {
      *v = r;
      return true;
    }
  }
  return false;
}

// protobuf wire helpers
void pb_varint(std::string* s, int field, uint64_t v) {
  put_varint(s, (uint64_t)(field << 3) | 0);
  put_varint(s, v);
}
void pb_bytes(std::string* s, int field, const std::string& b) {
  put_varint(s, (uint64_t)(field << 3) | 2);
  put_varint(s, b.size());
  s->append(b);
}
void pb_fixed32(std::string* s, int field, uint32_t v) {
  put_varint(s, (uint64_t)(field << 3) | 5);
  put_fixed32(s, v);
}

std::string header_proto() {
  std::string version;
  pb_varint(&version, 1, 1);  // producer = kTensorBundleVersion
  std::string s;
  pb_varint(&s, 1, 1);        // num_shards
  // endianness LITTLE = 0 (default, omitted)
  pb_bytes(&s, 3, version);
  return s;
}

std::string entry_proto(int dtype, const std::vector<int64_t>& shape, int64_t offset, int64_t size, uint32_t crc) {
  std::string shp;
  for (int64_t d : shape) {
    std::string dim;
    pb_varint(&dim, 1, (uint64_t)d);
    pb_bytes(&shp, 2, dim);
  }
  std::string s;
  pb_varint(&s, 1, (uint64_t)dtype);
  pb_bytes(&s, 2, shp);
  // shard_id = 0 omitted
  if (offset) pb_varint(&s, 4, (uint64_t)offset);
  if (size) pb_varint(&s, 5, (uint64_t)size);
  pb_fixed32(&s, 6, crc);
  return s;
}

struct Entry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard = 0;
  int64_t offset = 0, size = 0;
  uint32_t crc = 0;
};

bool parse_entry(const std::string& v, Entry* e) {
  const char* p = v.data();
  const char* end = p + v.size();
  while (p < end) {
    uint64_t tag;
    if (!get_varint(p, end, &tag)) return false;
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (wt == 0) {
      uint64_t x;
      if (!get_varint(p, end, &x)) return false;
      if (field == 1) e->dtype = (int)x;
      else if (field == 3) e->shard = (int)x;
      else if (field == 4) e->offset = (int64_t)x;
      else if (field == 5) e->size = (int64_t)x;
    } else if (wt == 2) {
      uint64_t n;
      if (!get_varint(p, end, &n) || p + n > end) return false;
      if (field == 2) {
        const char* q = p;
        const char* qe = p + n;
        while (q < qe) {
          uint64_t t2;
          if (!get_varint(q, qe, &t2)) return false;
          if ((t2 >> 3) == 2 && (t2 & 7) == 2) {
            uint64_t dn;
            if (!get_varint(q, qe, &dn)) return false;
            const char* r = q;
            const char* re = q + dn;
            int64_t size = 0;
            while (r < re) {
              uint64_t t3;
              if (!get_varint(r, re, &t3)) return false;
              if ((t3 & 7) == 0) {
                uint64_t x;
                if (!get_varint(r, re, &x)) return false;
                if ((t3 >> 3) == 1) size = (int64_t)x;
              } else if ((t3 & 7) == 2) {
                uint64_t sl;
                if (!get_varint(r, re, &sl)) return false;
                r += sl;
              } else {
                return false;
              }
            }
            e->shape.push_back(size);
            q = re;
          } else if ((t2 & 7) == 0) {
            uint64_t x;
            if (!get_varint(q, qe, &x)) return false;
          } else {
            return false;
          }
        }
      }
      p += n;
    } else if (wt == 5) {
      if (p + 4 > end) return false;
      uint32_t x;
      memcpy(&x, p, 4);
      p += 4;
      if (field == 6) e->crc = x;
    } else if (wt == 1) {
      p += 8;
    } else {
      return false;
    }
  }
  return true;
}

// ------------------------------------------------------------------ SSTable writer
struct BlockBuilder {
  int interval;
  std::string buf;
  std::vector<uint32_t> restarts{0};
  int counter = 0;
  std::string last_key;
  bool empty = true;
  explicit BlockBuilder(int iv) : interval(iv) {}
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < interval) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    put_varint(&buf, shared);
    put_varint(&buf, key.size() - shared);
    put_varint(&buf, value.size());
    buf.append(key.data() + shared, key.size() - shared);
    buf.append(value);
    last_key = key;
    ++counter;
    empty = false;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(&out, r);
    put_fixed32(&out, (uint32_t)restarts.size());
    return out;
  }
  size_t estimate() const { return buf.size() + restarts.size() * 4 + 4; }
};

struct TableWriter {
  std::string file;
  BlockBuilder data{kRestartInterval};
  BlockBuilder index{1};
  std::string pending_last_key;
  bool pending = false;
  uint64_t pending_off = 0, pending_size = 0;

  void write_block(const std::string& contents, uint64_t* off, uint64_t* size) {
    *off = file.size();
    *size = contents.size();
    file.append(contents);
    const char type = 0;  // kNoCompression
    uint32_t crc = crc32c(contents.data(), contents.size());
    crc = crc32c_extend(crc, &type, 1);
    file.push_back(type);
    put_fixed32(&file, crc32c_mask(crc));
  }
  static std::string handle(uint64_t off, uint64_t size) {
    std::string h;
    put_varint(&h, off);
    put_varint(&h, size);
    return h;
  }
  void flush_data() {
    if (data.empty) return;
    uint64_t off, size;
    write_block(data.finish(), &off, &size);
    index.add(data.last_key, handle(off, size));
    data = BlockBuilder(kRestartInterval);
  }
  void add(const std::string& k, const std::string& v) {
    data.add(k, v);
    if (data.estimate() >= kBlockSize) flush_data();
  }
  std::string finish() {
    flush_data();
    uint64_t moff, msize, ioff, isize;
    BlockBuilder meta(kRestartInterval);
    write_block(meta.finish(), &moff, &msize);
    write_block(index.finish(), &ioff, &isize);
    std::string footer = handle(moff, msize) + handle(ioff, isize);
    footer.resize(40, '\0');
    put_fixed64(&footer, kMagic);
    file.append(footer);
    return file;
  }
};

// ------------------------------------------------------------------ SSTable reader
bool read_file(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out->resize((size_t)n);
  bool ok = n == 0 || fread(&(*out)[0], 1, (size_t)n, f) == (size_t)n;
  fclose(f);
  return ok;
}

bool block_entries(const std::string& file, uint64_t off, uint64_t size,
                   std::vector<std::pair<std::string, std::string>>* out) {
  if (off + size + 5 > file.size()) return false;
  const char* b = file.data() + off;
  // verify trailer crc
  uint32_t stored;
  memcpy(&stored, b + size + 1, 4);
  uint32_t crc = crc32c(b, size);
  crc = crc32c_extend(crc, b + size, 1);
  if (crc32c_unmask(stored) != crc) return false;
  if (b[size] != 0) return false;  // compressed blocks unsupported
  if (size < 4) return false;
  uint32_t nres;
  memcpy(&nres, b + size - 4, 4);
  const size_t data_end = size - 4 - (size_t)nres * 4;
  const char* p = b;
  const char* end = b + data_end;
  std::string key;
  while (p < end) {
    uint64_t shared, nonshared, vlen;
    if (!get_varint(p, end, &shared) || !get_varint(p, end, &nonshared) || !get_varint(p, end, &vlen)) return false;
    if (shared > key.size() || p + nonshared + vlen > end) return false;
    key.resize(shared);
    key.append(p, nonshared);
    p += nonshared;
    out->emplace_back(key, std::string(p, vlen));
    p += vlen;
  }
  return true;
}

struct Bundle {
  std::string prefix;
  std::string data;  // data shard
  std::vector<std::string> names;
  std::map<std::string, Entry> entries;
  int num_shards = 1;
};

bool load_bundle(const std::string& prefix, Bundle* B) {
  std::string idx;
  if (!read_file(prefix + ".index", &idx) || idx.size() < 48) return false;
  uint64_t magic;
  memcpy(&magic, idx.data() + idx.size() - 8, 8);
  if (magic != kMagic) return false;
  const char* p = idx.data() + idx.size() - 48;
  const char* end = idx.data() + idx.size() - 8;
  uint64_t moff, msize, ioff, isize;
  if (!get_varint(p, end, &moff) || !get_varint(p, end, &msize) || !get_varint(p, end, &ioff) ||
      !get_varint(p, end, &isize))
    return false;
  std::vector<std::pair<std::string, std::string>> index;
  if (!block_entries(idx, ioff, isize, &index)) return false;
  for (auto& kv : index) {
    const char* q = kv.second.data();
    const char* qe = q + kv.second.size();
    uint64_t boff, bsize;
    if (!get_varint(q, qe, &boff) || !get_varint(q, qe, &bsize)) return false;
    std::vector<std::pair<std::string, std::string>> rows;
    if (!block_entries(idx, boff, bsize, &rows)) return false;
    for (auto& r : rows) {
      if (r.first.empty()) continue;  // header
      Entry e;
      if (!parse_entry(r.second, &e)) return false;
      B->names.push_back(r.first);
      B->entries[r.first] = e;
    }
  }
  B->prefix = prefix;
  return read_file(prefix + ".data-00000-of-00001", &B->data);
}

// Entry checksum of a DT_STRING tensor's data bytes, TF's string layout: the data is
// [varint64 len_0 .. len_{n-1}][masked crc32c of the lengths][string bytes]; the checksums run over the
// lengths as little-endian uint32 (uint64 above 4 GiB), NOT over the varint bytes, then the 4-byte length
// checksum, then the string bytes.  Returns false when the bytes do not parse as n strings.
bool string_tensor_crc(const char* d, size_t size, int64_t n, uint32_t* out) {
  size_t i = 0, total = 0;
  uint32_t crc = 0;
  for (int64_t k = 0; k < n; ++k) {
    uint64_t len = 0;
    int shift = 0;
    for (;;) {
      if (i >= size || shift > 63) return false;
      const uint8_t b = (uint8_t)d[i++];
      len |= (uint64_t)(b & 0x7f) << shift;
      shift += 7;
      if (!(b & 0x80)) break;
    }
    if (len <= 0xffffffffull) {
      const uint32_t l32 = (uint32_t)len;
      crc = crc32c_extend(crc, &l32, 4);
    } else {
      crc = crc32c_extend(crc, &len, 8);
    }
    total += (size_t)len;
  }
  if (i + 4 + total != size) return false;
  crc = crc32c_extend(crc, d + i, 4);            // the stored (masked) length checksum
  crc = crc32c_extend(crc, d + i + 4, total);     // the string bytes
  *out = crc32c_mask(crc);
  return true;
}

constexpr int kDtString = 7;

int64_t num_elements(const std::vector<int64_t>& shape) {
  int64_t n = 1;
  for (int64_t d : shape) n *= d;
  return n;
}

}  // namespace

// dtypes follow TF DataType: 1 float, 2 double, 3 int32, 4 uint8, 9 int64, 14 bfloat16, 19 half.
TDE_API int tde_bundle_write(const char* prefix, int n, const char** names, const int* dtypes, const int* ranks,
                             const long long* shapes_flat, const void** datas, const long long* nbytes) {
  std::vector<int> order(n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return strcmp(names[a], names[b]) < 0; });
  std::vector<size_t> shape_off(n);
  size_t so = 0;
  for (int i = 0; i < n; ++i) {
    shape_off[i] = so;
    so += (size_t)ranks[i];
  }
  std::string data;
  TableWriter tw;
  tw.add("", header_proto());
  for (int k = 0; k < n; ++k) {
    const int i = order[k];
    if (k > 0 && strcmp(names[order[k - 1]], names[i]) == 0) return -3;  // duplicate key
    const int64_t off = (int64_t)data.size();
    data.append((const char*)datas[i], (size_t)nbytes[i]);
    std::vector<int64_t> shape(shapes_flat + shape_off[i], shapes_flat + shape_off[i] + ranks[i]);
    uint32_t crc = 0;
    if (dtypes[i] == kDtString) {
      if (!string_tensor_crc((const char*)datas[i], (size_t)nbytes[i], num_elements(shape), &crc)) return -4;
    } else {
      crc = crc32c_mask(crc32c(datas[i], (size_t)nbytes[i]));
    }
    tw.add(names[i], entry_proto(dtypes[i], shape, off, nbytes[i], crc));
  }
  const std::string index = tw.finish();
  const std::string p(prefix);
  auto write_atomic = [](const std::string& path, const std::string& bytes) {
    const std::string tmp = path + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    bool ok = bytes.empty() || fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    ok = (fflush(f) == 0) && ok;
    fclose(f);
    return ok && rename(tmp.c_str(), path.c_str()) == 0;
  };
  // data first, index last: a reader never sees an index pointing at missing data
  if (!write_atomic(p + ".data-00000-of-00001", data)) return -1;
  if (!write_atomic(p + ".index", index)) return -2;
  return 0;
}

TDE_API void* tde_bundle_open(const char* prefix) {
  auto* b = new Bundle();
  if (!load_bundle(prefix, b)) {
    delete b;
    return nullptr;
  }
  return b;
}

TDE_API void tde_bundle_close(void* h) { delete (Bundle*)h; }

TDE_API int tde_bundle_count(void* h) { return (int)((Bundle*)h)->names.size(); }

// Describes entry i: name (NUL-terminated, truncated to cap), dtype, rank, shape (<= 16 dims), byte size.
TDE_API int tde_bundle_entry(void* h, int i, char* name, int cap, int* dtype, int* rank, long long* shape,
                             long long* nbytes) {
  auto* B = (Bundle*)h;
  if (i < 0 || i >= (int)B->names.size()) return -1;
  const std::string& nm = B->names[i];
  const Entry& e = B->entries[nm];
  snprintf(name, (size_t)cap, "%s", nm.c_str());
  *dtype = e.dtype;
  *rank = (int)e.shape.size();
  for (size_t d = 0; d < e.shape.size() && d < 16; ++d) shape[d] = e.shape[d];
  *nbytes = e.size;
  return 0;
}

// Copies tensor bytes; verifies the entry crc32c (string tensors: TF's length/bytes layout, see
// string_tensor_crc). Returns 0, -1 missing, -2 size, -3 crc mismatch.
TDE_API int tde_bundle_read(void* h, const char* name, void* out, long long cap) {
  auto* B = (Bundle*)h;
  auto it = B->entries.find(name);
  if (it == B->entries.end()) return -1;
  const Entry& e = it->second;
  if (e.size > cap || (size_t)(e.offset + e.size) > B->data.size()) return -2;
  const char* src = B->data.data() + e.offset;
  if (e.dtype == kDtString) {
    uint32_t crc = 0;
    if (!string_tensor_crc(src, (size_t)e.size, num_elements(e.shape), &crc) || crc != e.crc) return -3;
  } else if (crc32c_mask(crc32c(src, (size_t)e.size)) != e.crc) {
    return -3;
  }
  memcpy(out, src, (size_t)e.size);
  return 0;
}
