// Native real-data input pipeline core (the tf_cnn_benchmarks `--data_dir` path:
// preprocessing.py + datasets.py of the engine the reference drives with
// `--data_dir=... --data_name=imagenet`, /root/reference/benchmark-scripts/
// run-tf-sing-ucx-openmpi.sh:19,80-81; SURVEY.md §2.2 "preprocessing.py + datasets.py").
//
// What lives here (host C++, no GPU code):
//   * TFRecord framing: [u64 len][u32 masked crc32c(len)][data][u32 masked crc32c(data)],
//     CRC-32C via the SSE4.2 crc32 instruction (table fallback), reader + writer;
//   * a wire-format parser / encoder for tf.train.Example (Features map of
//     bytes_list / float_list / int64_list) -- only what ImageNet shards carry;
//   * JPEG header probing (SOFn marker -> height, width, components) so crop windows are
//     chosen without decoding;
//   * sample_distorted_bounding_box with TF's training-crop semantics (random aspect ratio and
//     area, min_object_covered against one of the labelled boxes, whole image on failure) and
//     the eval central crop;
//   * a Prefetcher: reader threads over this rank's shards (file i -> rank i % world), a
//     shuffle pool, epoch looping, and next_batch() that hands back (jpeg bytes, label, crop
//     window, flip) with the GIL released while it waits.
// JPEG entropy decoding stays in the Python layer (Pillow releases the GIL); resize / flip /
// normalise / NHWC-bf16 packing is the HIP kernel `preprocess_images` (csrc/kernels/data.hip).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace hcbdata {

// ------------------------------------------------------------------ CRC-32C (Castagnoli)
static uint32_t g_crc_tab[8][256];
static bool g_crc_hw = false;

static void crc_init() {
  static std::once_flag once;
  std::call_once(once, [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      g_crc_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int t = 1; t < 8; ++t) g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 0xff];
#if defined(__x86_64__)
    g_crc_hw = __builtin_cpu_supports("sse4.2");
#endif
  });
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) static uint32_t crc32c_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}
#endif

static uint32_t crc32c_sw(uint32_t crc, const uint8_t* p, size_t n) {
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= crc;
    crc = g_crc_tab[7][lo & 0xff] ^ g_crc_tab[6][(lo >> 8) & 0xff] ^ g_crc_tab[5][(lo >> 16) & 0xff] ^
          g_crc_tab[4][lo >> 24] ^ g_crc_tab[3][hi & 0xff] ^ g_crc_tab[2][(hi >> 8) & 0xff] ^
          g_crc_tab[1][(hi >> 16) & 0xff] ^ g_crc_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) crc = (crc >> 8) ^ g_crc_tab[0][(crc ^ *p++) & 0xff];
  return crc;
}

uint32_t crc32c(const void* data, size_t n) {
  crc_init();
  const uint8_t* p = static_cast<const uint8_t*>(data);
#if defined(__x86_64__)
  if (g_crc_hw) return ~crc32c_hw(~0u, p, n);
#endif
  return ~crc32c_sw(~0u, p, n);
}

static inline uint32_t masked_crc(const void* data, size_t n) {
  const uint32_t c = crc32c(data, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// ------------------------------------------------------------------ TFRecord files
class RecordReader {
 public:
  RecordReader(const std::string& path, bool verify) : path_(path), verify_(verify) {
    f_ = std::fopen(path.c_str(), "rb");
    if (!f_) throw std::runtime_error("tfrecord: cannot open " + path);
    std::setvbuf(f_, nullptr, _IOFBF, 1 << 20);
  }
  ~RecordReader() {
    if (f_) std::fclose(f_);
  }
  // false at a clean end of file; throws on truncation / CRC mismatch
  bool next(std::string& out) {
    uint8_t hdr[12];
    const size_t got = std::fread(hdr, 1, 12, f_);
    if (got == 0) return false;
    if (got != 12) throw std::runtime_error("tfrecord: truncated header in " + path_);
    uint64_t len;
    uint32_t lcrc;
    std::memcpy(&len, hdr, 8);
    std::memcpy(&lcrc, hdr + 8, 4);
    if (verify_ && masked_crc(hdr, 8) != lcrc) throw std::runtime_error("tfrecord: length CRC mismatch in " + path_);
    if (len > (1ull << 31)) throw std::runtime_error("tfrecord: record too large in " + path_);
    out.resize(len);
    uint32_t dcrc;
    if (std::fread(&out[0], 1, len, f_) != len || std::fread(&dcrc, 1, 4, f_) != 4)
      throw std::runtime_error("tfrecord: truncated record in " + path_);
    if (verify_ && masked_crc(out.data(), len) != dcrc) throw std::runtime_error("tfrecord: data CRC mismatch in " + path_);
    return true;
  }

 private:
  std::string path_;
  bool verify_;
  FILE* f_ = nullptr;
};

class RecordWriter {
 public:
  explicit RecordWriter(const std::string& path) {
    f_ = std::fopen(path.c_str(), "wb");
    if (!f_) throw std::runtime_error("tfrecord: cannot create " + path);
  }
  ~RecordWriter() { close(); }
  void write(const std::string& data) {
    if (!f_) throw std::runtime_error("tfrecord: writer closed");
    const uint64_t len = data.size();
    const uint32_t lcrc = masked_crc(&len, 8), dcrc = masked_crc(data.data(), data.size());
    std::fwrite(&len, 8, 1, f_);
    std::fwrite(&lcrc, 4, 1, f_);
    std::fwrite(data.data(), 1, data.size(), f_);
    std::fwrite(&dcrc, 4, 1, f_);
  }
  void close() {
    if (f_) std::fclose(f_);
    f_ = nullptr;
  }

 private:
  FILE* f_ = nullptr;
};

// ------------------------------------------------------------------ tf.train.Example wire format
struct Feature {
  int kind = 0;  // 1 bytes, 2 float, 3 int64
  std::vector<std::string> bytes;
  std::vector<float> floats;
  std::vector<int64_t> ints;
};
using Features = std::map<std::string, Feature>;

struct Cursor {
  const uint8_t* p;
  const uint8_t* e;
  bool done() const { return p >= e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) throw std::runtime_error("example: truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("example: varint too long");
  }
  Cursor sub() {
    const uint64_t n = varint();
    if (n > (uint64_t)(e - p)) throw std::runtime_error("example: length past end");
    Cursor c{p, p + n};
    p += n;
    return c;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) p += 8;
    else if (wt == 2) sub();
    else if (wt == 5) p += 4;
    else throw std::runtime_error("example: unsupported wire type");
    if (p > e) throw std::runtime_error("example: field past end");
  }
};

static void parse_feature(Cursor c, Feature& f) {
  while (!c.done()) {
    const uint64_t tag = c.varint();
    const int field = (int)(tag >> 3), wt = (int)(tag & 7);
    if (wt != 2 || field < 1 || field > 3) {
      c.skip(wt);
      continue;
    }
    Cursor list = c.sub();
    f.kind = field;
    while (!list.done()) {
      const uint64_t t2 = list.varint();
      const int f2 = (int)(t2 >> 3), w2 = (int)(t2 & 7);
      if (f2 != 1) {
        list.skip(w2);
        continue;
      }
      if (field == 1 && w2 == 2) {
        Cursor b = list.sub();
        f.bytes.emplace_back(reinterpret_cast<const char*>(b.p), b.e - b.p);
      } else if (field == 2 && w2 == 2) {  // packed floats
        Cursor b = list.sub();
        const size_t n = (b.e - b.p) / 4;
        const size_t o = f.floats.size();
        f.floats.resize(o + n);
        std::memcpy(f.floats.data() + o, b.p, n * 4);
      } else if (field == 2 && w2 == 5) {
        float v;
        if (list.e - list.p < 4) throw std::runtime_error("example: truncated float");
        std::memcpy(&v, list.p, 4);
        list.p += 4;
        f.floats.push_back(v);
      } else if (field == 3 && w2 == 2) {  // packed varints
        Cursor b = list.sub();
        while (!b.done()) f.ints.push_back((int64_t)b.varint());
      } else if (field == 3 && w2 == 0) {
        f.ints.push_back((int64_t)list.varint());
      } else {
        list.skip(w2);
      }
    }
  }
}

Features parse_example(const std::string& rec) {
  Features out;
  Cursor c{reinterpret_cast<const uint8_t*>(rec.data()), reinterpret_cast<const uint8_t*>(rec.data()) + rec.size()};
  while (!c.done()) {
    const uint64_t tag = c.varint();
    if ((tag >> 3) != 1 || (tag & 7) != 2) {
      c.skip((int)(tag & 7));
      continue;
    }
    Cursor feats = c.sub();
    while (!feats.done()) {
      const uint64_t t1 = feats.varint();
      if ((t1 >> 3) != 1 || (t1 & 7) != 2) {
        feats.skip((int)(t1 & 7));
        continue;
      }
      Cursor entry = feats.sub();
      std::string key;
      Feature f;
      while (!entry.done()) {
        const uint64_t t2 = entry.varint();
        if ((t2 >> 3) == 1 && (t2 & 7) == 2) {
          Cursor k = entry.sub();
          key.assign(reinterpret_cast<const char*>(k.p), k.e - k.p);
        } else if ((t2 >> 3) == 2 && (t2 & 7) == 2) {
          parse_feature(entry.sub(), f);
        } else {
          entry.skip((int)(t2 & 7));
        }
      }
      out[key] = std::move(f);
    }
  }
  return out;
}

static void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
static void put_len(std::string& s, int field, const std::string& body) {
  put_varint(s, ((uint64_t)field << 3) | 2);
  put_varint(s, body.size());
  s += body;
}

std::string encode_example(const Features& feats) {
  std::string features;
  for (const auto& kv : feats) {
    const Feature& f = kv.second;
    std::string list;
    if (f.kind == 1) {
      for (const auto& b : f.bytes) put_len(list, 1, b);
    } else if (f.kind == 2) {
      std::string packed(reinterpret_cast<const char*>(f.floats.data()), f.floats.size() * 4);
      put_len(list, 1, packed);
    } else {
      std::string packed;
      for (int64_t v : f.ints) put_varint(packed, (uint64_t)v);
      put_len(list, 1, packed);
    }
    std::string feature;
    put_len(feature, f.kind, list);
    std::string entry;
    put_len(entry, 1, kv.first);
    put_len(entry, 2, feature);
    put_len(features, 1, entry);
  }
  std::string ex;
  put_len(ex, 1, features);
  return ex;
}

// ------------------------------------------------------------------ JPEG header probe
// Returns false if no SOFn marker is found (not a JPEG / corrupt); h, w, components otherwise.
bool jpeg_dims(const std::string& b, int& h, int& w, int& comps) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(b.data());
  const size_t n = b.size();
  if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return false;
  size_t i = 2;
  while (i + 4 <= n) {
    if (p[i] != 0xFF) {
      ++i;
      continue;
    }
    const uint8_t m = p[i + 1];
    if (m == 0xFF) {
      ++i;
      continue;
    }
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) {
      i += 2;
      continue;
    }
    const size_t seg = ((size_t)p[i + 2] << 8) | p[i + 3];
    const bool sof = (m >= 0xC0 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC;
    if (sof) {
      if (i + 9 >= n) return false;
      h = (p[i + 5] << 8) | p[i + 6];
      w = (p[i + 7] << 8) | p[i + 8];
      comps = p[i + 9];
      return h > 0 && w > 0;
    }
    if (m == 0xDA || m == 0xD9) return false;  // scan started without a frame header
    i += 2 + seg;
  }
  return false;
}

// ------------------------------------------------------------------ crop windows
struct Box {
  float ymin, xmin, ymax, xmax;  // normalised
};
struct Window {
  int y, x, h, w;
};

// One try of TF's training crop: an integer crop of aspect `ar` whose area fraction lies in
// [area_lo, area_hi] of the image, placed uniformly at random.
static bool random_crop(int H, int W, float area_lo, float area_hi, float ar, std::mt19937_64& rng, Window& out) {
  const double min_area = area_lo * (double)W * H, max_area = area_hi * (double)W * H;
  int height = (int)std::lround(std::sqrt(min_area / ar));
  int max_height = (int)std::lround(std::sqrt(max_area / ar));
  if (std::lround(max_height * ar) > W) max_height = (int)((W + 0.5 - 1e-7) / ar);
  max_height = std::min(max_height, H);
  if (height > max_height) height = max_height;
  if (height < max_height) height += (int)(rng() % (uint64_t)(max_height - height + 1));
  int width = (int)std::lround(height * ar);
  double area = (double)width * height;
  if (area < min_area) {
    height += 1;
    width = (int)std::lround(height * ar);
    area = (double)width * height;
  }
  if (area < min_area || area > max_area || width > W || height > H || width <= 0 || height <= 0) return false;
  out.y = (int)(rng() % (uint64_t)(H - height + 1));
  out.x = (int)(rng() % (uint64_t)(W - width + 1));
  out.h = height;
  out.w = width;
  return true;
}

Window distorted_crop(int H, int W, const std::vector<Box>& boxes, float min_cov, float ar_lo, float ar_hi, float area_lo,
                      float area_hi, int attempts, std::mt19937_64& rng) {
  std::uniform_real_distribution<float> u01(0.f, 1.f);
  Box b{0.f, 0.f, 1.f, 1.f};
  if (!boxes.empty()) b = boxes[rng() % boxes.size()];
  const float by0 = b.ymin * H, bx0 = b.xmin * W, by1 = b.ymax * H, bx1 = b.xmax * W;
  const float barea = std::max(0.f, by1 - by0) * std::max(0.f, bx1 - bx0);
  for (int a = 0; a < attempts; ++a) {
    const float ar = ar_lo + (ar_hi - ar_lo) * u01(rng);
    Window win;
    if (!random_crop(H, W, area_lo, area_hi, ar, rng, win)) continue;
    if (barea <= 0.f) return win;
    const float iy = std::max(0.f, std::min(by1, (float)(win.y + win.h)) - std::max(by0, (float)win.y));
    const float ix = std::max(0.f, std::min(bx1, (float)(win.x + win.w)) - std::max(bx0, (float)win.x));
    if (iy * ix / barea >= min_cov) return win;
  }
  return Window{0, 0, H, W};
}

Window central_crop(int H, int W, float fraction) {
  const int h = std::max(1, (int)(H * fraction)), w = std::max(1, (int)(W * fraction));
  return Window{(H - h) / 2, (W - w) / 2, h, w};
}

// ------------------------------------------------------------------ prefetcher
struct Sample {
  std::string jpeg;
  std::vector<Box> boxes;
  int64_t label;
  Window win;
  int flip;
  int h, w;
};

struct PrefetchConfig {
  std::vector<std::string> files;
  int rank = 0, world = 1;
  int threads = 4;
  int shuffle_buffer = 2048;
  int capacity = 8192;
  uint64_t seed = 0;
  bool train = true;
  bool loop = true;
  bool verify_crc = true;
  float min_object_covered = 0.1f, ar_lo = 0.75f, ar_hi = 1.33f, area_lo = 0.05f, area_hi = 1.0f;
  int attempts = 100;
  float central_fraction = 0.875f;
  int label_offset = 0;
};

class Prefetcher {
 public:
  explicit Prefetcher(PrefetchConfig cfg) : cfg_(std::move(cfg)) {
    rng_.seed(cfg_.seed * 0x9E3779B97F4A7C15ull + (uint64_t)cfg_.rank);
    crop_rng_.seed(cfg_.seed * 0xD1B54A32D192ED03ull + (uint64_t)cfg_.rank + 1);
    if (cfg_.files.empty()) throw std::runtime_error("prefetcher: no input files");
    // shards of this rank (file i -> rank i % world); with fewer files than ranks every rank
    // reads every file and keeps record j when j % world == rank
    for (size_t i = 0; i < cfg_.files.size(); ++i)
      if ((int)(i % cfg_.world) == cfg_.rank || (int)cfg_.files.size() < cfg_.world) mine_.push_back(cfg_.files[i]);
    record_stride_ = (int)cfg_.files.size() < cfg_.world ? cfg_.world : 1;
    const int T = std::max(1, std::min<int>(cfg_.threads, (int)mine_.size()));
    for (int t = 0; t < T; ++t) workers_.emplace_back([this, t, T] { run(t, T); });
  }
  ~Prefetcher() { stop(); }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_put_.notify_all();
    cv_get_.notify_all();
    for (auto& th : workers_)
      if (th.joinable()) th.join();
    workers_.clear();
  }

  // Blocks until n samples are available (or the data is exhausted without looping).
  std::vector<Sample> next(int n) {
    std::vector<Sample> out;
    out.reserve(n);
    std::unique_lock<std::mutex> lk(mu_);
    while ((int)out.size() < n) {
      cv_get_.wait(lk, [&] {
        return stop_ || !error_.empty() || (int)pool_.size() >= std::min(cfg_.shuffle_buffer, cfg_.capacity) ||
               (finished_ == (int)workers_.size() && !pool_.empty()) || finished_ == (int)workers_.size();
      });
      if (!error_.empty()) throw std::runtime_error(error_);
      if (pool_.empty()) {
        if (stop_ || finished_ == (int)workers_.size()) break;
        continue;
      }
      // shuffle: take a random element of the pool (train), FIFO otherwise
      size_t k = 0;
      if (cfg_.train && pool_.size() > 1) k = rng_() % pool_.size();
      std::swap(pool_[k], pool_.back());
      out.push_back(std::move(pool_.back()));
      pool_.pop_back();
      cv_put_.notify_one();
    }
    lk.unlock();
    for (auto& s : out) finish(s);
    return out;
  }

  int64_t records_read() const { return records_.load(); }
  int epochs() const { return epoch_.load(); }
  size_t num_files() const { return mine_.size(); }

 private:
  void finish(Sample& s) {
    if (cfg_.train) {
      s.win = distorted_crop(s.h, s.w, s.boxes, cfg_.min_object_covered, cfg_.ar_lo, cfg_.ar_hi, cfg_.area_lo,
                             cfg_.area_hi, cfg_.attempts, crop_rng_);
      s.flip = (int)(crop_rng_() & 1);
    } else {
      s.win = central_crop(s.h, s.w, cfg_.central_fraction);
      s.flip = 0;
    }
  }

  void run(int t, int T) {
    std::string rec;
    std::mt19937_64 order_rng(cfg_.seed * 7919 + (uint64_t)cfg_.rank * 104729 + t);
    try {
      for (int ep = 0;; ++ep) {
        std::vector<std::string> files;
        for (size_t i = t; i < mine_.size(); i += T) files.push_back(mine_[i]);
        if (cfg_.train) std::shuffle(files.begin(), files.end(), order_rng);
        for (const auto& path : files) {
          RecordReader rd(path, cfg_.verify_crc);
          int64_t j = 0;
          while (rd.next(rec)) {
            if (record_stride_ > 1 && (j++ % record_stride_) != cfg_.rank) continue;
            Sample s;
            Features f = parse_example(rec);
            auto it = f.find("image/encoded");
            if (it == f.end() || it->second.bytes.empty())
              throw std::runtime_error("prefetcher: record without image/encoded in " + path);
            s.jpeg = std::move(it->second.bytes[0]);
            auto lb = f.find("image/class/label");
            s.label = (lb != f.end() && !lb->second.ints.empty()) ? lb->second.ints[0] + cfg_.label_offset : -1;
            int comps = 3;
            if (!jpeg_dims(s.jpeg, s.h, s.w, comps)) {
              // not a JPEG (a few ImageNet files are PNG / CMYK): fall back to the stored dims
              auto hh = f.find("image/height"), ww = f.find("image/width");
              s.h = (hh != f.end() && !hh->second.ints.empty()) ? (int)hh->second.ints[0] : 0;
              s.w = (ww != f.end() && !ww->second.ints.empty()) ? (int)ww->second.ints[0] : 0;
            }
            // labelled object boxes (normalised [ymin, xmin, ymax, xmax]) for the training crop
            auto y0 = f.find("image/object/bbox/ymin"), x0 = f.find("image/object/bbox/xmin");
            auto y1 = f.find("image/object/bbox/ymax"), x1 = f.find("image/object/bbox/xmax");
            if (y0 != f.end() && x0 != f.end() && y1 != f.end() && x1 != f.end()) {
              const size_t nb = std::min(std::min(y0->second.floats.size(), x0->second.floats.size()),
                                         std::min(y1->second.floats.size(), x1->second.floats.size()));
              for (size_t q = 0; q < nb; ++q)
                s.boxes.push_back(Box{y0->second.floats[q], x0->second.floats[q], y1->second.floats[q], x1->second.floats[q]});
            }
            s.win = Window{0, 0, s.h, s.w};
            s.flip = 0;
            push(std::move(s));
            if (stopped()) return;
          }
        }
        epoch_.fetch_add(1);
        if (!cfg_.loop) break;
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> g(mu_);
      if (error_.empty()) error_ = e.what();
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      ++finished_;
    }
    cv_get_.notify_all();
  }

  bool stopped() {
    std::lock_guard<std::mutex> g(mu_);
    return stop_;
  }

  void push(Sample&& s) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_put_.wait(lk, [&] { return stop_ || (int)pool_.size() < cfg_.capacity; });
    if (stop_) return;
    pool_.push_back(std::move(s));
    records_.fetch_add(1);
    lk.unlock();
    cv_get_.notify_one();
  }

  PrefetchConfig cfg_;
  std::vector<std::string> mine_;
  int record_stride_ = 1;
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_put_, cv_get_;
  std::vector<Sample> pool_;
  bool stop_ = false;
  int finished_ = 0;
  std::string error_;
  std::mt19937_64 rng_{0x9E3779B97F4A7C15ull};
  std::mt19937_64 crop_rng_{0xD1B54A32D192ED03ull};
  std::atomic<int64_t> records_{0};
  std::atomic<int> epoch_{0};
};

}  // namespace hcbdata

// ------------------------------------------------------------------ Python bindings
using namespace hcbdata;

static py::object feature_to_py(const Feature& f) {
  if (f.kind == 1) {
    py::list l;
    for (const auto& b : f.bytes) l.append(py::bytes(b));
    return l;
  }
  if (f.kind == 2) return py::cast(f.floats);
  return py::cast(f.ints);
}

static Feature py_to_feature(const py::handle& v) {
  Feature f;
  py::list items;
  if (py::isinstance<py::bytes>(v) || py::isinstance<py::str>(v) || py::isinstance<py::int_>(v) ||
      py::isinstance<py::float_>(v))
    items.append(v);
  else
    items = py::reinterpret_steal<py::list>(PySequence_List(v.ptr()));
  if (!items) throw py::error_already_set();
  if (items.size() == 0) {
    f.kind = 3;
    return f;
  }
  py::handle first = items[0];
  if (py::isinstance<py::bytes>(first) || py::isinstance<py::str>(first)) {
    f.kind = 1;
    for (auto x : items) f.bytes.push_back(py::isinstance<py::str>(x) ? x.cast<std::string>() : std::string(py::bytes(x.cast<py::bytes>())));
  } else if (py::isinstance<py::float_>(first)) {
    f.kind = 2;
    for (auto x : items) f.floats.push_back(x.cast<float>());
  } else {
    f.kind = 3;
    for (auto x : items) f.ints.push_back(x.cast<int64_t>());
  }
  return f;
}

PYBIND11_MODULE(_hcb_data, m) {
  m.doc() = "native TFRecord / tf.Example / crop-window / prefetch core of the real-data input pipeline";
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c(s.data(), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return masked_crc(s.data(), s.size());
  });
  m.def("parse_example", [](py::bytes b) {
    std::string s = b;
    Features f = parse_example(s);
    py::dict d;
    for (const auto& kv : f) d[py::str(kv.first)] = feature_to_py(kv.second);
    return d;
  });
  m.def("encode_example", [](py::dict d) {
    Features f;
    for (auto kv : d) f[kv.first.cast<std::string>()] = py_to_feature(kv.second);
    return py::bytes(encode_example(f));
  });
  m.def("jpeg_dims", [](py::bytes b) -> py::object {
    std::string s = b;
    int h = 0, w = 0, c = 0;
    if (!jpeg_dims(s, h, w, c)) return py::none();
    return py::make_tuple(h, w, c);
  });
  m.def(
      "distorted_crop",
      [](int H, int W, std::vector<std::tuple<float, float, float, float>> boxes, uint64_t seed, float min_cov, float ar_lo,
         float ar_hi, float area_lo, float area_hi, int attempts) {
        std::vector<Box> bx;
        for (auto& t : boxes) bx.push_back(Box{std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t)});
        std::mt19937_64 rng(seed);
        Window w = distorted_crop(H, W, bx, min_cov, ar_lo, ar_hi, area_lo, area_hi, attempts, rng);
        return py::make_tuple(w.y, w.x, w.h, w.w);
      },
      py::arg("H"), py::arg("W"), py::arg("boxes") = std::vector<std::tuple<float, float, float, float>>{},
      py::arg("seed") = 0, py::arg("min_object_covered") = 0.1f, py::arg("ar_lo") = 0.75f, py::arg("ar_hi") = 1.33f,
      py::arg("area_lo") = 0.05f, py::arg("area_hi") = 1.0f, py::arg("attempts") = 100);
  m.def("central_crop", [](int H, int W, float frac) {
    Window w = central_crop(H, W, frac);
    return py::make_tuple(w.y, w.x, w.h, w.w);
  });

  py::class_<RecordReader>(m, "RecordReader")
      .def(py::init<const std::string&, bool>(), py::arg("path"), py::arg("verify_crc") = true)
      .def("next", [](RecordReader& r) -> py::object {
        std::string s;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = r.next(s);
        }
        if (!ok) return py::none();
        return py::bytes(s);
      });
  py::class_<RecordWriter>(m, "RecordWriter")
      .def(py::init<const std::string&>())
      .def("write", [](RecordWriter& w, py::bytes b) { w.write(std::string(b)); })
      .def("close", &RecordWriter::close);

  py::class_<Prefetcher>(m, "Prefetcher")
      .def(py::init([](std::vector<std::string> files, int rank, int world, int threads, int shuffle_buffer, int capacity,
                       uint64_t seed, bool train, bool loop, bool verify_crc, int label_offset, float central_fraction) {
             PrefetchConfig c;
             c.files = std::move(files);
             c.rank = rank;
             c.world = world;
             c.threads = threads;
             c.shuffle_buffer = shuffle_buffer;
             c.capacity = std::max(capacity, shuffle_buffer);
             c.seed = seed;
             c.train = train;
             c.loop = loop;
             c.verify_crc = verify_crc;
             c.label_offset = label_offset;
             c.central_fraction = central_fraction;
             return new Prefetcher(std::move(c));
           }),
           py::arg("files"), py::arg("rank") = 0, py::arg("world") = 1, py::arg("threads") = 4,
           py::arg("shuffle_buffer") = 2048, py::arg("capacity") = 8192, py::arg("seed") = 0, py::arg("train") = true,
           py::arg("loop") = true, py::arg("verify_crc") = true, py::arg("label_offset") = 0,
           py::arg("central_fraction") = 0.875f)
      .def("next",
           [](Prefetcher& p, int n) {
             std::vector<Sample> v;
             {
               py::gil_scoped_release nogil;
               v = p.next(n);
             }
             py::list out;
             for (auto& s : v)
               out.append(py::make_tuple(py::bytes(s.jpeg), s.label, py::make_tuple(s.win.y, s.win.x, s.win.h, s.win.w),
                                         s.flip, py::make_tuple(s.h, s.w)));
             return out;
           })
      .def("stop", [](Prefetcher& p) {
        py::gil_scoped_release nogil;
        p.stop();
      })
      .def_property_readonly("records_read", &Prefetcher::records_read)
      .def_property_readonly("epochs", &Prefetcher::epochs)
      .def_property_readonly("num_files", &Prefetcher::num_files);
}
