// llmctl native host runtime (C++17, pybind11): paged-KV block allocator, continuous-batching
// admission core, and a memory-mapped token loader with a background prefetch thread.
//
// These are the host-side hot paths of serving and training input: they run every engine
// step / every batch, so they are native rather than Python (the reference has no runtime
// of its own: its KV "manager" is a Python dict, server.py:57-87, and its data is a
// hard-coded list of strings, engine.py:147-156).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

// ============================================================================ block allocator
// Fixed-size KV blocks in one preallocated HBM pool; reference-counted so prefix blocks can
// be shared (fork / prefix caching); LIFO free list keeps recently freed (cache-warm) blocks hot.
class BlockAllocator {
 public:
  BlockAllocator(int64_t num_blocks, int64_t block_size) : num_blocks_(num_blocks), block_size_(block_size) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("num_blocks and block_size must be > 0");
    ref_.assign(num_blocks, 0);
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  }
  int64_t allocate() {
    if (free_.empty()) return -1;
    int64_t b = free_.back();
    free_.pop_back();
    ref_[b] = 1;
    return b;
  }
  std::vector<int64_t> allocate_n(int64_t n) {
    if ((int64_t)free_.size() < n) return {};
    std::vector<int64_t> out(n);
    for (int64_t i = 0; i < n; ++i) out[i] = allocate();
    return out;
  }
  void incref(int64_t b) {
    check(b);
    if (ref_[b] <= 0) throw std::runtime_error("incref of a free block");
    ++ref_[b];
  }
  // returns true when the block went back to the free list
  bool free(int64_t b) {
    check(b);
    if (ref_[b] <= 0) throw std::runtime_error("double free of KV block " + std::to_string(b));
    if (--ref_[b] == 0) {
      free_.push_back(b);
      return true;
    }
    return false;
  }
  int64_t num_free() const { return (int64_t)free_.size(); }
  int64_t num_blocks() const { return num_blocks_; }
  int64_t block_size() const { return block_size_; }
  int32_t refcount(int64_t b) const {
    check(b);
    return ref_[b];
  }

 private:
  void check(int64_t b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("block id out of range");
  }
  int64_t num_blocks_, block_size_;
  std::vector<int32_t> ref_;
  std::vector<int64_t> free_;
};

// ============================================================================ sequence KV tables
// Per-sequence block tables + token counts on top of the allocator; produces the int32
// block-table matrix and int64 slot mapping the paged-attention kernels consume.
class KVManager {
 public:
  KVManager(int64_t num_blocks, int64_t block_size) : alloc_(num_blocks, block_size), bs_(block_size) {}

  int64_t blocks_needed(int64_t tokens) const { return (tokens + bs_ - 1) / bs_; }

  bool can_allocate(int64_t tokens) const { return blocks_needed(tokens) <= alloc_.num_free(); }

  // reserve blocks for a new sequence holding `tokens` tokens; returns false if out of memory
  bool add_sequence(int64_t seq, int64_t tokens) {
    if (tables_.count(seq)) throw std::runtime_error("sequence already registered");
    auto blocks = alloc_.allocate_n(blocks_needed(std::max<int64_t>(tokens, 1)));
    if (blocks.empty()) return false;  // (a 0-token sequence reserves one block too)
    tables_[seq] = {std::move(blocks), tokens};
    return true;
  }

  // new sequence of `tokens` tokens whose first blocks are the (already cached, shared) `prefix`
  // blocks: each gets one more reference, the rest are allocated; false (nothing changed) if OOM
  bool add_sequence_shared(int64_t seq, int64_t tokens, const std::vector<int64_t>& prefix) {
    if (tables_.count(seq)) throw std::runtime_error("sequence already registered");
    const int64_t need = blocks_needed(std::max<int64_t>(tokens, 1));
    if ((int64_t)prefix.size() > need) throw std::invalid_argument("prefix longer than the sequence");
    const int64_t fresh = need - (int64_t)prefix.size();
    if (fresh > alloc_.num_free()) return false;
    Table t;
    t.tokens = tokens;
    for (auto b : prefix) {
      alloc_.incref(b);
      t.blocks.push_back(b);
    }
    for (int64_t i = 0; i < fresh; ++i) t.blocks.push_back(alloc_.allocate());
    tables_[seq] = std::move(t);
    return true;
  }

  // a reference held outside any sequence (the prefix cache); decref returns true when freed
  void incref_block(int64_t b) { alloc_.incref(b); }
  bool decref_block(int64_t b) { return alloc_.free(b); }
  int32_t refcount(int64_t b) const { return alloc_.refcount(b); }

  // make room for one more token; returns its flat slot (block*bs + offset) or -1 if OOM
  int64_t append_token(int64_t seq) {
    auto& t = get(seq);
    int64_t pos = t.tokens;
    if (pos / bs_ >= (int64_t)t.blocks.size()) {
      int64_t b = alloc_.allocate();
      if (b < 0) return -1;
      t.blocks.push_back(b);
    }
    t.tokens = pos + 1;
    return t.blocks[pos / bs_] * bs_ + pos % bs_;
  }

  int64_t slot(int64_t seq, int64_t pos) {
    auto& t = get(seq);
    if (pos >= (int64_t)t.blocks.size() * bs_) throw std::out_of_range("position beyond reserved blocks");
    return t.blocks[pos / bs_] * bs_ + pos % bs_;
  }

  // share all full blocks of `src` with a new sequence `dst` (copy-on-write prefix sharing)
  void fork(int64_t src, int64_t dst) {
    if (tables_.count(dst)) throw std::runtime_error("sequence already registered");
    auto& s = get(src);
    Table t;
    t.tokens = s.tokens;
    for (auto b : s.blocks) {
      alloc_.incref(b);
      t.blocks.push_back(b);
    }
    tables_[dst] = std::move(t);
  }

  void free_sequence(int64_t seq) {
    auto it = tables_.find(seq);
    if (it == tables_.end()) return;
    for (auto b : it->second.blocks) alloc_.free(b);
    tables_.erase(it);
  }

  int64_t num_tokens(int64_t seq) { return get(seq).tokens; }
  std::vector<int64_t> block_table(int64_t seq) { return get(seq).blocks; }

  // [n, max_blocks] int32 block table (padded with 0) for a batch of sequences
  py::array_t<int32_t> block_tables(const std::vector<int64_t>& seqs, int64_t max_blocks) {
    py::array_t<int32_t> out({(py::ssize_t)seqs.size(), (py::ssize_t)max_blocks});
    auto m = out.mutable_unchecked<2>();
    for (size_t i = 0; i < seqs.size(); ++i) {
      auto& t = get(seqs[i]);
      if ((int64_t)t.blocks.size() > max_blocks) throw std::runtime_error("max_blocks too small");
      for (int64_t j = 0; j < max_blocks; ++j) m(i, j) = j < (int64_t)t.blocks.size() ? (int32_t)t.blocks[j] : 0;
    }
    return out;
  }

  // flat slots for positions [start, start+count) of a sequence (prefill)
  py::array_t<int64_t> slots(int64_t seq, int64_t start, int64_t count) {
    py::array_t<int64_t> out(count);
    auto m = out.mutable_unchecked<1>();
    for (int64_t i = 0; i < count; ++i) m(i) = slot(seq, start + i);
    return out;
  }

  int64_t num_free_blocks() const { return alloc_.num_free(); }
  int64_t num_blocks() const { return alloc_.num_blocks(); }
  int64_t num_sequences() const { return (int64_t)tables_.size(); }
  double usage() const { return 1.0 - (double)alloc_.num_free() / (double)alloc_.num_blocks(); }

 private:
  struct Table {
    std::vector<int64_t> blocks;
    int64_t tokens = 0;
  };
  Table& get(int64_t seq) {
    auto it = tables_.find(seq);
    if (it == tables_.end()) throw std::out_of_range("unknown sequence " + std::to_string(seq));
    return it->second;
  }
  BlockAllocator alloc_;
  int64_t bs_;
  std::unordered_map<int64_t, Table> tables_;
};

// ============================================================================ token loader
// Packed next-token samples from a flat uint16/uint32 token file (mmap), DP-strided epoch
// permutation (seed, epoch), and a prefetch thread that keeps `depth` batches ready.
class TokenLoader {
 public:
  TokenLoader(const std::string& path, int itemsize, int64_t seq_len, int64_t batch, int64_t rank, int64_t world,
              uint64_t seed, int depth = 4)
      : itemsize_(itemsize), S_(seq_len), B_(batch), rank_(rank), world_(world), seed_(seed), depth_(depth) {
    if (itemsize != 2 && itemsize != 4) throw std::invalid_argument("itemsize must be 2 or 4");
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path);
    struct stat st;
    fstat(fd_, &st);
    bytes_ = st.st_size;
    n_tokens_ = bytes_ / itemsize_;
    base_ = (const uint8_t*)mmap(nullptr, bytes_, PROT_READ, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    madvise((void*)base_, bytes_, MADV_RANDOM);
    n_samples_ = (n_tokens_ - 1) / S_;
    if (n_samples_ < world_ * B_) throw std::runtime_error("token file too small for one global batch");
    per_rank_ = n_samples_ / world_;
    make_perm();
    worker_ = std::thread([this] { this->run(); });
  }
  ~TokenLoader() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    munmap((void*)base_, bytes_);
    ::close(fd_);
  }

  py::array_t<int64_t> next() {
    std::vector<int64_t> batch;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return !queue_.empty() || stop_; });
      batch = std::move(queue_.front().data);
      cur_epoch_ = queue_.front().epoch;
      cur_pos_ = queue_.front().pos_after;
      queue_.pop_front();
    }
    cv_.notify_all();
    py::array_t<int64_t> out({(py::ssize_t)B_, (py::ssize_t)(S_ + 1)});
    std::memcpy(out.mutable_data(), batch.data(), batch.size() * sizeof(int64_t));
    return out;
  }

  std::pair<int64_t, int64_t> position() const { return {cur_epoch_, cur_pos_}; }

  void seek(int64_t epoch, int64_t pos) {
    std::lock_guard<std::mutex> g(mu_);
    epoch_ = epoch;
    pos_ = pos;
    make_perm();
    queue_.clear();
    cv_.notify_all();
  }

  int64_t num_samples() const { return n_samples_; }

 private:
  struct Item {
    std::vector<int64_t> data;
    int64_t epoch, pos_after;
  };
  void make_perm() {
    perm_.resize(n_samples_);
    std::iota(perm_.begin(), perm_.end(), 0);
    std::mt19937_64 g(seed_ * 1000003ULL + (uint64_t)epoch_ * 7919ULL);
    std::shuffle(perm_.begin(), perm_.end(), g);
  }
  int64_t tok(int64_t i) const {
    return itemsize_ == 2 ? (int64_t)((const uint16_t*)base_)[i] : (int64_t)((const uint32_t*)base_)[i];
  }
  void run() {
    while (true) {
      std::vector<int64_t> data((size_t)(B_ * (S_ + 1)));
      int64_t e, p;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return (int)queue_.size() < depth_ || stop_; });
        if (stop_) return;
        if (pos_ + B_ > per_rank_) {
          ++epoch_;
          pos_ = 0;
          make_perm();
        }
        for (int64_t b = 0; b < B_; ++b) {
          int64_t sample = perm_[(size_t)((pos_ + b) * world_ + rank_)];
          int64_t off = sample * S_;
          for (int64_t t = 0; t <= S_; ++t) data[(size_t)(b * (S_ + 1) + t)] = tok(off + t);
        }
        pos_ += B_;
        e = epoch_;
        p = pos_;
        queue_.push_back({std::move(data), e, p});
      }
      cv_.notify_all();
    }
  }
  int itemsize_;
  int64_t S_, B_, rank_, world_;
  uint64_t seed_;
  int depth_;
  int fd_ = -1;
  size_t bytes_ = 0;
  const uint8_t* base_ = nullptr;
  int64_t n_tokens_ = 0, n_samples_ = 0, per_rank_ = 0;
  int64_t epoch_ = 0, pos_ = 0, cur_epoch_ = 0, cur_pos_ = 0;
  std::vector<int64_t> perm_;
  std::deque<Item> queue_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread worker_;
  bool stop_ = false;
};

// ============================================================================ byte-level indexer
// text (one document per line / jsonl "text") -> uint16 tokens + uint64 document offsets
py::tuple index_bytes(const std::string& text_path, const std::string& bin_path, const std::string& idx_path,
                      bool jsonl) {
  FILE* in = fopen(text_path.c_str(), "rb");
  if (!in) throw std::runtime_error("cannot open " + text_path);
  FILE* ob = fopen(bin_path.c_str(), "wb");
  FILE* oi = fopen(idx_path.c_str(), "wb");
  if (!ob || !oi) throw std::runtime_error("cannot open outputs");
  std::vector<uint16_t> buf;
  std::string line;
  char chunk[1 << 16];
  uint64_t ntok = 0, ndocs = 0;
  std::vector<uint64_t> offsets{0};
  auto flush_doc = [&](const std::string& doc) {
    std::string body = doc;
    if (jsonl) {  // minimal extraction of "text": "..."
      auto k = doc.find("\"text\"");
      if (k == std::string::npos) return;
      auto q = doc.find('"', doc.find(':', k) + 1);
      std::string out;
      for (size_t i = q + 1; i < doc.size(); ++i) {
        char c = doc[i];
        if (c == '\\' && i + 1 < doc.size()) {
          char n = doc[++i];
          if (n == 'u' && i + 4 < doc.size()) {
            uint32_t cp = std::stoul(doc.substr(i + 1, 4), nullptr, 16);
            i += 4;
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 < doc.size() && doc[i + 1] == '\\' && doc[i + 2] == 'u') {
              uint32_t lo = std::stoul(doc.substr(i + 3, 4), nullptr, 16);
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              i += 6;
            }
            if (cp < 0x80) {
              out.push_back(char(cp));
            } else if (cp < 0x800) {
              out.push_back(char(0xC0 | (cp >> 6)));
              out.push_back(char(0x80 | (cp & 0x3F)));
            } else if (cp < 0x10000) {
              out.push_back(char(0xE0 | (cp >> 12)));
              out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
              out.push_back(char(0x80 | (cp & 0x3F)));
            } else {
              out.push_back(char(0xF0 | (cp >> 18)));
              out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
              out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
              out.push_back(char(0x80 | (cp & 0x3F)));
            }
          } else {
            out.push_back(n == 'n' ? '\n' : n == 't' ? '\t' : n == 'r' ? '\r' : n == 'b' ? '\b' : n == 'f' ? '\f' : n);
          }
        } else if (c == '"') {
          break;
        } else {
          out.push_back(c);
        }
      }
      body = out;
    }
    buf.clear();
    for (unsigned char c : body) buf.push_back(c);
    buf.push_back(0);
    fwrite(buf.data(), sizeof(uint16_t), buf.size(), ob);
    ntok += buf.size();
    offsets.push_back(ntok);
    ++ndocs;
  };
  while (size_t n = fread(chunk, 1, sizeof(chunk), in)) {
    for (size_t i = 0; i < n; ++i) {
      if (chunk[i] == '\n') {
        if (!line.empty()) flush_doc(line);
        line.clear();
      } else {
        line.push_back(chunk[i]);
      }
    }
  }
  if (!line.empty()) flush_doc(line);
  fwrite(offsets.data(), sizeof(uint64_t), offsets.size(), oi);
  fclose(in);
  fclose(ob);
  fclose(oi);
  return py::make_tuple(ntok, ndocs);
}

PYBIND11_MODULE(_llmctl_native, m) {
  m.doc() = "llmctl native host runtime (KV block allocator, token loader, indexer)";
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int64_t, int64_t>())
      .def("allocate", &BlockAllocator::allocate)
      .def("allocate_n", &BlockAllocator::allocate_n)
      .def("incref", &BlockAllocator::incref)
      .def("free", &BlockAllocator::free)
      .def("refcount", &BlockAllocator::refcount)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size);
  py::class_<KVManager>(m, "KVManager")
      .def(py::init<int64_t, int64_t>())
      .def("blocks_needed", &KVManager::blocks_needed)
      .def("can_allocate", &KVManager::can_allocate)
      .def("add_sequence", &KVManager::add_sequence)
      .def("append_token", &KVManager::append_token)
      .def("slot", &KVManager::slot)
      .def("fork", &KVManager::fork)
      .def("add_sequence_shared", &KVManager::add_sequence_shared)
      .def("incref_block", &KVManager::incref_block)
      .def("decref_block", &KVManager::decref_block)
      .def("refcount", &KVManager::refcount)
      .def("free_sequence", &KVManager::free_sequence)
      .def("num_tokens", &KVManager::num_tokens)
      .def("block_table", &KVManager::block_table)
      .def("block_tables", &KVManager::block_tables)
      .def("slots", &KVManager::slots)
      .def_property_readonly("num_free_blocks", &KVManager::num_free_blocks)
      .def_property_readonly("num_blocks", &KVManager::num_blocks)
      .def_property_readonly("num_sequences", &KVManager::num_sequences)
      .def("usage", &KVManager::usage);
  py::class_<TokenLoader>(m, "TokenLoader")
      .def(py::init<const std::string&, int, int64_t, int64_t, int64_t, int64_t, uint64_t, int>(), py::arg("path"),
           py::arg("itemsize"), py::arg("seq_len"), py::arg("batch"), py::arg("rank"), py::arg("world"),
           py::arg("seed"), py::arg("depth") = 4)
      .def("next", &TokenLoader::next)
      .def("position", &TokenLoader::position)
      .def("seek", &TokenLoader::seek)
      .def_property_readonly("num_samples", &TokenLoader::num_samples);
  m.def("index_bytes", &index_bytes, py::arg("text_path"), py::arg("bin_path"), py::arg("idx_path"),
        py::arg("jsonl") = false);
}
