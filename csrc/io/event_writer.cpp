// TensorBoard event files: the summaries the reference's
// Estimator writes every save_summary_steps=100 (mnist_keras_distributed.py:246)
// and the global_step/sec of log_step_count_steps=100 (:247).
//
// File: events.out.tfevents.<time>.<host>, a TFRecord stream:
//   uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)
// Records are tensorflow.Event protos, hand-encoded:
//   Event { double wall_time = 1; int64 step = 2; string file_version = 3; Summary summary = 5; }
//   Summary { repeated Value value = 1; }  Value { string tag = 1; float simple_value = 2; }
// Stock TensorBoard reads these files unchanged.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <string>

#define TDE_API extern "C" __attribute__((visibility("default")))

namespace tde_host {
uint32_t crc32c(const void* data, size_t n);
uint32_t crc32c_mask(uint32_t crc);
uint32_t crc32c_unmask(uint32_t m);
}  // namespace tde_host

namespace {

void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)(v | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}

void tag(std::string* s, int field, int wt) { put_varint(s, (uint64_t)((field << 3) | wt)); }

std::string event_header(double wall_time, int64_t step) {
  std::string e;
  tag(&e, 1, 1);
  e.append((const char*)&wall_time, 8);
  if (step) {
    tag(&e, 2, 0);
    put_varint(&e, (uint64_t)step);
  }
  return e;
}

struct EventFile {
  FILE* f = nullptr;
  std::mutex mu;
  bool write_record(const std::string& data) {
    std::lock_guard<std::mutex> g(mu);
    const uint64_t len = data.size();
    const uint32_t lcrc = tde_host::crc32c_mask(tde_host::crc32c(&len, 8));
    const uint32_t dcrc = tde_host::crc32c_mask(tde_host::crc32c(data.data(), data.size()));
    return fwrite(&len, 8, 1, f) == 1 && fwrite(&lcrc, 4, 1, f) == 1 &&
           (data.empty() || fwrite(data.data(), 1, data.size(), f) == data.size()) && fwrite(&dcrc, 4, 1, f) == 1;
  }
};

}  // namespace

TDE_API void* tde_events_open(const char* path) {
  FILE* f = fopen(path, "ab");
  if (!f) return nullptr;
  auto* e = new EventFile();
  e->f = f;
  return e;
}

TDE_API int tde_events_write_version(void* h, double wall_time) {
  std::string e = event_header(wall_time, 0);
  const std::string v = "brain.Event:2";
  tag(&e, 3, 2);
  put_varint(&e, v.size());
  e.append(v);
  return ((EventFile*)h)->write_record(e) ? 0 : -1;
}

// n scalar values (tags[i], values[i]) in one Event at `step`.
TDE_API int tde_events_write_scalars(void* h, double wall_time, long long step, int n, const char** tags,
                                     const float* values) {
  std::string summary;
  for (int i = 0; i < n; ++i) {
    std::string val;
    const size_t tl = strlen(tags[i]);
    tag(&val, 1, 2);
    put_varint(&val, tl);
    val.append(tags[i], tl);
    tag(&val, 2, 5);
    val.append((const char*)&values[i], 4);
    tag(&summary, 1, 2);
    put_varint(&summary, val.size());
    summary.append(val);
  }
  std::string e = event_header(wall_time, step);
  tag(&e, 5, 2);
  put_varint(&e, summary.size());
  e.append(summary);
  return ((EventFile*)h)->write_record(e) ? 0 : -1;
}

TDE_API int tde_events_write_raw(void* h, const void* data, long long n) {
  return ((EventFile*)h)->write_record(std::string((const char*)data, (size_t)n)) ? 0 : -1;
}

TDE_API int tde_events_flush(void* h) { return fflush(((EventFile*)h)->f); }

TDE_API void tde_events_close(void* h) {
  auto* e = (EventFile*)h;
  if (!e) return;
  fclose(e->f);
  delete e;
}

// Reader for tests/tools: iterate records of a TFRecord file, verifying both crcs.
// Returns number of records (or -k if record k is corrupt); copies record i into out if i >= 0.
TDE_API long long tde_tfrecord_scan(const char* path, long long want, void* out, long long cap,
                                    long long* out_len) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1000000;
  long long idx = 0;
  std::string buf;
  while (true) {
    uint64_t len;
    uint32_t lcrc, dcrc;
    if (fread(&len, 8, 1, f) != 1) break;
    if (fread(&lcrc, 4, 1, f) != 1 || tde_host::crc32c_mask(tde_host::crc32c(&len, 8)) != lcrc) {
      fclose(f);
      return -(idx + 1);
    }
    buf.resize(len);
    if ((len && fread(&buf[0], 1, len, f) != len) || fread(&dcrc, 4, 1, f) != 1 ||
        tde_host::crc32c_mask(tde_host::crc32c(buf.data(), len)) != dcrc) {
      fclose(f);
      return -(idx + 1);
    }
    if (idx == want && out) {
      memcpy(out, buf.data(), (size_t)(len < (uint64_t)cap ? len : (uint64_t)cap));
      if (out_len) *out_len = (long long)len;
    }
    ++idx;
  }
  fclose(f);
  return idx;
}
