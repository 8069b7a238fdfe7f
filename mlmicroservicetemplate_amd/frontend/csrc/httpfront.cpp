// Native HTTP/1.1 front end for the batched serving path (FRONTEND=native).
//
// Why: the Python front end (FastAPI/uvicorn) parses ~1k ResNet uploads/s per process while one
// MI355X engine retires ~37k images/s (profiles/r1_http_resnet50_workers_per_gpu.jsonl).  Here
// the whole per-request path is C++: epoll I/O threads accept, read and parse HTTP/1.1 +
// multipart, queue the raw pixels of a fixed-shape sample, and format the JSON responses;
// Python is entered once per BATCH (a dispatcher thread blocks in next_batch() with the GIL
// released, receives the batch memcpy'd straight into the engine slot's pinned host buffer,
// replays the hipGraph and hands back top-k arrays).
//
// Wire behaviour follows the reference service (reference src/server/main.py:52-140; SURVEY.md
// Appendix A): GET / -> ["MLMicroserviceTemplate is Running!"], GET /status 503 / 200 bodies,
// POST /predict multipart field `image_file` (missing -> 422, checked before readiness -> 503),
// CORS for the configured origins with credentials (main.py:21-38).  Requests the native side
// does not serve itself (non-raw images that need a decoder, /health, /metrics, /info, the legacy
// ?filename= flow, unknown routes) are queued to Python handler threads under a token.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <utility>
#include <vector>

#include "jpeg_coefs.h"

namespace py = pybind11;
using Clock = std::chrono::steady_clock;

namespace {

constexpr const char* ROOT_BODY = "[\"MLMicroserviceTemplate is Running!\"]";
constexpr const char* NOT_READY_BODY =
    "{\"status\":\"failure\",\"detail\":\"Model is not ready to receive predictions.\"}";
constexpr const char* READY_BODY =
    "{\"status\":\"success\",\"detail\":\"Model ready to receive prediction requests.\"}";
constexpr const char* OVERLOAD_BODY = "{\"status\":\"failure\",\"detail\":\"Server overloaded; retry later.\"}";
constexpr size_t MAX_HEAD = 64 * 1024;

const char* reason(int code) {
  switch (code) {
    case 200: return "OK";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 411: return "Length Required";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Status";
  }
}

bool ieq(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
  return true;
}

bool istarts(std::string_view s, std::string_view p) { return s.size() >= p.size() && ieq(s.substr(0, p.size()), p); }

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

void json_escape(std::string& out, std::string_view s) {
  out.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          out += b;
        } else {
          out.push_back((char)c);
        }
    }
  }
  out.push_back('"');
}

std::string failure_body(std::string_view detail) {
  std::string b = "{\"status\":\"failure\",\"detail\":";
  json_escape(b, detail);
  b += "}";
  return b;
}

// Value of `key` in a header parameter list such as `multipart/form-data; boundary="xyz"`.
std::string_view header_param(std::string_view h, std::string_view key) {
  size_t i = 0;
  while (i < h.size()) {
    size_t semi = h.find(';', i);
    std::string_view item = trim(h.substr(i, semi == std::string_view::npos ? std::string_view::npos : semi - i));
    size_t eq = item.find('=');
    if (eq != std::string_view::npos && ieq(trim(item.substr(0, eq)), key)) {
      std::string_view v = trim(item.substr(eq + 1));
      if (v.size() >= 2 && v.front() == '"' && v.back() == '"') v = v.substr(1, v.size() - 2);
      return v;
    }
    if (semi == std::string_view::npos) break;
    i = semi + 1;
  }
  return {};
}

struct Part {
  std::string_view name, filename, content_type, data;
};

// multipart/form-data body -> parts (views into `body`); false on malformed framing.
bool parse_multipart(std::string_view body, std::string_view boundary, std::vector<Part>& parts) {
  if (boundary.empty() || boundary.size() > 200) return false;
  std::string delim = "--";
  delim.append(boundary);
  size_t pos = body.find(delim);
  if (pos == std::string_view::npos) return false;
  pos += delim.size();
  std::string next = "\r\n";
  next += delim;
  for (;;) {
    if (body.substr(pos, 2) == "--") return true;  // closing delimiter
    if (body.substr(pos, 2) != "\r\n") return false;
    pos += 2;
    size_t hend = body.find("\r\n\r\n", pos);
    if (hend == std::string_view::npos) return false;
    Part p;
    std::string_view heads = body.substr(pos, hend - pos);
    size_t l = 0;
    while (l <= heads.size()) {
      size_t e = heads.find("\r\n", l);
      std::string_view line = heads.substr(l, e == std::string_view::npos ? std::string_view::npos : e - l);
      size_t colon = line.find(':');
      if (colon != std::string_view::npos) {
        std::string_view k = trim(line.substr(0, colon)), v = trim(line.substr(colon + 1));
        if (ieq(k, "content-disposition")) {
          p.name = header_param(v, "name");
          p.filename = header_param(v, "filename");
        } else if (ieq(k, "content-type")) {
          p.content_type = v;
        }
      }
      if (e == std::string_view::npos) break;
      l = e + 2;
    }
    size_t dstart = hend + 4;
    size_t dend = body.find(next, dstart);
    if (dend == std::string_view::npos) return false;
    p.data = body.substr(dstart, dend - dstart);
    parts.push_back(p);
    pos = dend + next.size();
  }
}

bool raw_content_type(std::string_view ct) {
  ct = trim(ct.substr(0, ct.find(';')));
  return ct.empty() || ieq(ct, "application/octet-stream") || ieq(ct, "application/x-rgb8");
}

// Hash tokenizer of models/bert.py:HashTokenizer for pure-ASCII texts, run on the I/O thread so a
// text request never touches Python: lowercase, split into [a-z0-9]+ runs and single other
// non-space characters (whitespace = Python's str.isspace() over ASCII: \t \n \v \f \r
// \x1c-\x1f and space), id = 1000 + crc32(token) % (vocab - 1000), framed by CLS / SEP and cut
// at max_len exactly as encode() does.  Non-ASCII texts go to the Python tokenizer (Unicode
// lowercasing / whitespace), so both paths give the same ids.
struct TextHash {
  int vocab = 0, max_len = 0, seq = 0, cls = 101, sep = 102;
};

uint32_t crc32_bytes(const char* p, size_t n) {
  static const auto table = [] {
    std::vector<uint32_t> t(256);
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[i] = c;
    }
    return t;
  }();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ (uint8_t)p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

inline bool ascii_space(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }
inline bool ascii_alnum(unsigned char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }

// -> false when the text is not pure ASCII (caller falls back to Python); else ids (truncated to seq)
bool hash_tokenize(std::string_view text, const TextHash& th, std::vector<int32_t>& ids) {
  for (unsigned char c : text)
    if (c >= 0x80) return false;
  ids.clear();
  ids.push_back(th.cls);
  const uint32_t span = (uint32_t)(th.vocab - 1000);
  std::string w;
  size_t i = 0;
  while (i < text.size()) {
    const unsigned char c = text[i];
    if (ascii_space(c)) { ++i; continue; }
    w.clear();
    if (ascii_alnum(c)) {
      while (i < text.size() && ascii_alnum((unsigned char)text[i])) {
        unsigned char d = text[i++];
        w.push_back((char)((d >= 'A' && d <= 'Z') ? d + 32 : d));
      }
    } else {
      w.push_back((char)c);
      ++i;
    }
    ids.push_back((int32_t)(1000 + crc32_bytes(w.data(), w.size()) % span));
    if ((int)ids.size() >= th.max_len - 1) break;
  }
  ids.push_back(th.sep);
  if ((int)ids.size() > th.seq) ids.resize(th.seq);
  return true;
}

struct ReqRef {
  int thread = -1;
  uint64_t conn = 0;
  bool keep_alive = true;
  std::string origin;  // an allowed CORS origin to echo, or empty
  Clock::time_point t0;
};

struct Pending {  // one fixed-shape sample waiting for a batch
  ReqRef ref;
  std::string body;  // owns the bytes; the sample is body[off, off + sample_bytes)
  size_t off = 0;
};

struct DecodeItem {
  uint64_t token = 0;
  std::string data;
  std::string ctype;
};

struct PyRequest {
  uint64_t token = 0;
  std::string method, path, query;
  std::vector<std::pair<std::string, std::string>> headers;
  std::string body;
};

struct Outgoing {
  uint64_t conn;
  std::string bytes;
  bool close;
};

struct Buf {  // growable byte buffer with a consumed prefix
  std::unique_ptr<char[]> p;
  size_t cap = 0, beg = 0, end = 0;
  size_t size() const { return end - beg; }
  const char* data() const { return p.get() + beg; }
  void consume(size_t n) {
    beg += n;
    if (beg >= end) beg = end = 0;
  }
  void reserve_tail(size_t n) {  // ensure n writable bytes after `end`
    if (cap - end >= n) return;
    if (beg > 0 && cap - size() >= n) {
      memmove(p.get(), p.get() + beg, size());
      end -= beg;
      beg = 0;
      return;
    }
    size_t ncap = std::max(cap * 2, size() + n);
    std::unique_ptr<char[]> q(new char[ncap]);
    if (size()) memcpy(q.get(), p.get() + beg, size());
    end -= beg;
    beg = 0;
    p = std::move(q);
    cap = ncap;
  }
  void append(const char* s, size_t n) {
    reserve_tail(n);
    memcpy(p.get() + end, s, n);
    end += n;
  }
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  Buf in, out;
  bool waiting = false;      // a request was dispatched; its response has not arrived yet
  bool close_after = false;  // close once `out` drains
  bool peer_eof = false;
  bool sent_continue = false;
};

struct Head {
  std::string_view method, target, path, query;
  std::string_view content_type, origin, connection, expect, transfer_encoding, acr_method, acr_headers;
  long long content_length = -1;
  bool http10 = false;
  size_t head_len = 0;
};

struct IoThread {
  int idx = 0;
  int ep = -1, efd = -1;
  std::thread th;
  std::mutex mu;
  std::vector<Outgoing> outbox;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;
};

class Server {
 public:
  struct Config {
    std::string host = "0.0.0.0";
    int port = 0;
    int listen_fd = -1;
    int io_threads = 4;
    long long sample_bytes = 0;
    // false: every upload goes through the Python preprocess (a text model's packed sample must
    // never be taken verbatim from a client body that happens to have the same size)
    bool raw_samples = true;
    TextHash text_hash;  // vocab > 0: tokenise ASCII texts in C++ into packed (2*seq+1) int32 rows
    int max_batch = 32;
    int max_wait_us = 2000;
    int max_queue = 4096;
    long long max_upload = 32 << 20;
    std::string form_field = "image_file";
    std::vector<std::string> cors_origins;
    double request_timeout_s = 30.0;
    bool python_decode = true;
    // samples are GPU image containers (jpeg_coefs.h): raw RGB uploads are wrapped, baseline JPEGs
    // Huffman-decoded here on the I/O thread; anything else goes to the Python decode threads
    bool image_container = false;
  };

  explicit Server(Config c) : cfg_(std::move(c)) {}
  ~Server() { stop(); }

  int port() const { return bound_port_; }

  void start() {
    if (running_.exchange(true)) return;
    if (cfg_.listen_fd >= 0) {
      lfd_ = cfg_.listen_fd;
    } else {
      lfd_ = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (lfd_ < 0) throw std::runtime_error("socket() failed");
      int one = 1;
      setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)cfg_.port);
      if (inet_pton(AF_INET, cfg_.host.c_str(), &a.sin_addr) != 1) a.sin_addr.s_addr = htonl(INADDR_ANY);
      if (bind(lfd_, (sockaddr*)&a, sizeof a) != 0 || listen(lfd_, 4096) != 0) {
        int e = errno;
        close(lfd_);
        lfd_ = -1;
        running_ = false;
        throw std::runtime_error(std::string("bind/listen failed: ") + strerror(e));
      }
      own_lfd_ = true;
    }
    fcntl(lfd_, F_SETFL, fcntl(lfd_, F_GETFL) | O_NONBLOCK);
    sockaddr_in b{};
    socklen_t bl = sizeof b;
    getsockname(lfd_, (sockaddr*)&b, &bl);
    bound_port_ = ntohs(b.sin_port);
    int n = std::max(1, cfg_.io_threads);
    for (int i = 0; i < n; ++i) {
      auto t = std::make_unique<IoThread>();
      t->idx = i;
      t->ep = epoll_create1(EPOLL_CLOEXEC);
      t->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
      epoll_event ev{};
      // own socket: wake one I/O thread per connection.  A socket inherited from the launcher is
      // shared by every serving process on the port: wake them all (new connections are rare with
      // keep-alive) so the accepting process is random instead of always the same waiter.
      ev.events = own_lfd_ ? (EPOLLIN | EPOLLEXCLUSIVE) : EPOLLIN;
      ev.data.u64 = 0;
      epoll_ctl(t->ep, EPOLL_CTL_ADD, lfd_, &ev);
      ev.events = EPOLLIN;
      ev.data.u64 = 1;
      epoll_ctl(t->ep, EPOLL_CTL_ADD, t->efd, &ev);
      threads_.push_back(std::move(t));
    }
    for (auto& t : threads_) {
      IoThread* tp = t.get();
      tp->th = std::thread([this, tp] { io_loop(*tp); });
    }
  }

  void stop() {
    if (!running_.exchange(false)) return;
    {
      std::lock_guard<std::mutex> g(qmu_);
      stopping_ = true;
    }
    qcv_.notify_all();
    dcv_.notify_all();
    rcv_.notify_all();
    for (auto& t : threads_) {
      uint64_t one = 1;
      (void)!write(t->efd, &one, sizeof one);
    }
    for (auto& t : threads_) {
      if (t->th.joinable()) t->th.join();
      for (auto& kv : t->conns) close(kv.second->fd);
      t->conns.clear();
      close(t->ep);
      close(t->efd);
    }
    if (own_lfd_ && lfd_ >= 0) close(lfd_);
    lfd_ = -1;
  }

  void set_ready(bool r, const std::string& err) {
    std::lock_guard<std::mutex> g(state_mu_);
    ready_ = r;
    init_error_ = err;
  }

  void set_labels(const std::vector<std::string>& labels) {
    std::vector<std::string> enc;
    enc.reserve(labels.size());
    for (auto& l : labels) {
      std::string e;
      json_escape(e, l);
      enc.push_back(std::move(e));
    }
    std::lock_guard<std::mutex> g(state_mu_);
    labels_json_ = std::move(enc);
  }

  // ---- batch path --------------------------------------------------------------------------
  // Blocks until a batch is due: up to `cap` samples, at most max_wait_us after the oldest
  // pending one arrived (the scheduler/batcher.py DynamicBatcher rule).  Copies the samples
  // into `dst` (the engine slot's pinned host buffer) and returns (batch_id, n); n == 0 on
  // timeout / shutdown.  Several consumers may wait concurrently (one per in-flight slot).
  std::pair<uint64_t, int> next_batch(char* dst, size_t dst_bytes, int cap, int timeout_ms) {
    const size_t sb = (size_t)cfg_.sample_bytes;
    if (sb == 0) throw std::runtime_error("next_batch: server was built without a sample size");
    cap = (int)std::min<long long>(cap, (long long)(dst_bytes / sb));
    if (cap <= 0) throw std::runtime_error("next_batch: buffer smaller than one sample");
    std::vector<Pending> take;
    {
      std::unique_lock<std::mutex> lk(qmu_);
      auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
      while (pending_.empty() && !stopping_) {
        if (qcv_.wait_until(lk, deadline) == std::cv_status::timeout && pending_.empty()) return {0, 0};
      }
      if (stopping_) return {0, 0};
      for (;;) {  // wait for a full batch or the oldest sample's deadline
        if (pending_.empty() || stopping_) return {0, 0};  // another consumer took them
        auto due = pending_.front().ref.t0 + std::chrono::microseconds(cfg_.max_wait_us);
        if ((int)pending_.size() >= cap || Clock::now() >= due) break;
        qcv_.wait_until(lk, due);
      }
      const auto expire = Clock::now() - std::chrono::duration_cast<Clock::duration>(
                                             std::chrono::duration<double>(cfg_.request_timeout_s));
      while ((int)take.size() < cap && !pending_.empty()) {
        Pending p = std::move(pending_.front());
        pending_.pop_front();
        if (p.ref.t0 < expire) {  // queued past REQUEST_TIMEOUT_S
          reply(p.ref, 504, failure_body("Prediction timed out."));
          continue;
        }
        take.push_back(std::move(p));
      }
      if (!pending_.empty()) qcv_.notify_one();  // more work for another consumer
    }
    if (take.empty()) return {0, 0};
    std::vector<ReqRef> refs;
    refs.reserve(take.size());
    for (size_t i = 0; i < take.size(); ++i) {
      memcpy(dst + i * sb, take[i].body.data() + take[i].off, sb);
      refs.push_back(std::move(take[i].ref));
    }
    const int n = (int)refs.size();
    const uint64_t id = next_id_.fetch_add(1);
    {
      std::lock_guard<std::mutex> g(bmu_);
      batches_.emplace(id, std::move(refs));
    }
    n_batches_++;
    n_samples_ += n;
    return {id, n};
  }

  void complete_topk(uint64_t id, const float* vals, const int32_t* idx, int n, int k) {
    std::vector<ReqRef> refs = take_batch(id);
    if ((int)refs.size() != n) {
      for (auto& r : refs) reply(r, 500, failure_body("engine returned the wrong number of rows"));
      throw std::runtime_error("complete_topk: row count != batch size");
    }
    std::vector<std::string> labels;
    {
      std::lock_guard<std::mutex> g(state_mu_);
      labels = labels_json_;
    }
    for (int r = 0; r < n; ++r) {
      if (k > 0 && idx[r * k] < 0) {  // the GPU image decode flagged this upload (ids -1): as PIL's error
        reply(refs[r], 500, failure_body("ValueError: undecodable image"));
        continue;
      }
      std::string body = "{\"status\":\"success\",\"result\":{\"classes\":[";
      for (int j = 0; j < k; ++j) {
        if (j) body += ',';
        append_label(body, labels, idx[r * k + j]);
      }
      body += "],\"result\":{";
      for (int j = 0; j < k; ++j) {
        if (j) body += ',';
        append_label(body, labels, idx[r * k + j]);
        char num[40];
        snprintf(num, sizeof num, ":%.9g", (double)vals[r * k + j]);
        body += num;
      }
      body += "}}}";
      reply(refs[r], 200, body);
    }
  }

  void complete_json(uint64_t id, const std::vector<std::string>& results) {
    std::vector<ReqRef> refs = take_batch(id);
    if (results.size() != refs.size()) {
      for (auto& r : refs) reply(r, 500, failure_body("plugin returned the wrong number of results"));
      throw std::runtime_error("complete_json: result count != batch size");
    }
    for (size_t i = 0; i < results.size(); ++i) {
      std::string body = "{\"status\":\"success\",\"result\":";
      body += results[i];
      body += "}";
      reply(refs[i], 200, body);
    }
  }

  void fail_batch(uint64_t id, int code, const std::string& detail) {
    for (auto& r : take_batch(id)) reply(r, code, failure_body(detail));
  }

  // ---- Python-handled requests (image decode / generic routes) -------------------------------
  bool next_decode(int timeout_ms, DecodeItem& out) {
    std::unique_lock<std::mutex> lk(qmu_);
    dcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return stopping_ || !decode_q_.empty(); });
    if (decode_q_.empty() || stopping_) return false;
    out = std::move(decode_q_.front());
    decode_q_.pop_front();
    return true;
  }

  bool next_request(int timeout_ms, PyRequest& out) {
    std::unique_lock<std::mutex> lk(qmu_);
    rcv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return stopping_ || !req_q_.empty(); });
    if (req_q_.empty() || stopping_) return false;
    out = std::move(req_q_.front());
    req_q_.pop_front();
    return true;
  }

  // A decoded sample for a token from next_decode() / next_request(): joins the batch queue.
  bool submit_sample(uint64_t token, const char* data, size_t n) {
    ReqRef ref;
    if (!take_token(token, ref)) return false;
    if ((long long)n != cfg_.sample_bytes) {
      reply(ref, 500, failure_body("decoded sample has the wrong size"));
      return false;
    }
    Pending p;
    p.ref = std::move(ref);
    p.body.assign(data, n);
    enqueue_sample(std::move(p));
    return true;
  }

  bool respond(uint64_t token, int code, const std::string& body, const std::string& ctype,
               const std::vector<std::pair<std::string, std::string>>& headers) {
    ReqRef ref;
    if (!take_token(token, ref)) return false;
    std::string extra;
    for (auto& h : headers) {
      if (h.first.find_first_of("\r\n") != std::string::npos || h.second.find_first_of("\r\n") != std::string::npos)
        continue;  // no header injection
      extra += h.first + ": " + h.second + "\r\n";
    }
    reply(ref, code, body, ctype, extra);
    return true;
  }

  std::map<std::string, long long> stats() {
    std::map<std::string, long long> s;
    s["requests"] = n_requests_;
    s["batches"] = n_batches_;
    s["samples"] = n_samples_;
    s["rejected_overload"] = n_overload_;
    s["python_routed"] = n_python_;
    s["decode_routed"] = n_decode_;
    s["jpeg_native"] = n_jpeg_native_;
    s["text_hashed"] = n_text_hash_;
    s["connections_open"] = n_conns_;
    {
      std::lock_guard<std::mutex> g(qmu_);
      s["queue_depth"] = (long long)pending_.size();
    }
    std::lock_guard<std::mutex> g(cmu_);
    for (auto& kv : code_counts_) s["status_" + std::to_string(kv.first)] = kv.second;
    return s;
  }

 private:
  Config cfg_;
  std::atomic<bool> running_{false};
  int lfd_ = -1;
  bool own_lfd_ = false;
  int bound_port_ = 0;
  std::vector<std::unique_ptr<IoThread>> threads_;

  std::mutex state_mu_;
  bool ready_ = false;
  std::string init_error_;
  std::vector<std::string> labels_json_;

  std::mutex qmu_;  // pending_, decode_q_, req_q_, stopping_
  std::condition_variable qcv_, dcv_, rcv_;
  bool stopping_ = false;
  std::deque<Pending> pending_;
  std::deque<DecodeItem> decode_q_;
  std::deque<PyRequest> req_q_;

  std::mutex bmu_;
  std::unordered_map<uint64_t, std::vector<ReqRef>> batches_;
  std::mutex tmu_;
  std::unordered_map<uint64_t, ReqRef> tokens_;
  std::atomic<uint64_t> next_id_{1};
  std::atomic<uint64_t> next_conn_{2};  // 0 = listen socket, 1 = eventfd

  std::atomic<long long> n_jpeg_native_{0};
  std::atomic<long long> n_requests_{0}, n_batches_{0}, n_samples_{0}, n_overload_{0}, n_python_{0}, n_decode_{0}, n_text_hash_{0},
      n_conns_{0};
  std::mutex cmu_;
  std::map<int, long long> code_counts_;

  std::vector<ReqRef> take_batch(uint64_t id) {
    std::lock_guard<std::mutex> g(bmu_);
    auto it = batches_.find(id);
    if (it == batches_.end()) throw std::runtime_error("unknown batch id");
    std::vector<ReqRef> refs = std::move(it->second);
    batches_.erase(it);
    return refs;
  }

  bool take_token(uint64_t token, ReqRef& ref) {
    std::lock_guard<std::mutex> g(tmu_);
    auto it = tokens_.find(token);
    if (it == tokens_.end()) return false;
    ref = std::move(it->second);
    tokens_.erase(it);
    return true;
  }

  uint64_t new_token(ReqRef ref) {
    const uint64_t t = next_id_.fetch_add(1);
    std::lock_guard<std::mutex> g(tmu_);
    tokens_.emplace(t, std::move(ref));
    return t;
  }

  static void append_label(std::string& body, const std::vector<std::string>& labels, int i) {
    if (i >= 0 && i < (int)labels.size()) {
      body += labels[i];
    } else {
      body += "\"class_" + std::to_string(i) + "\"";
    }
  }

  void enqueue_sample(Pending p) {
    std::unique_lock<std::mutex> lk(qmu_);
    if ((int)pending_.size() >= cfg_.max_queue) {
      lk.unlock();
      n_overload_++;
      reply(p.ref, 503, OVERLOAD_BODY, "application/json", "retry-after: 1\r\n");
      return;
    }
    pending_.push_back(std::move(p));
    // wake a consumer on the first sample (it starts the max-wait clock) and once a full batch
    // is queued; in between the consumer sleeps until the oldest sample's deadline
    if (pending_.size() == 1 || (int)pending_.size() >= cfg_.max_batch) qcv_.notify_one();
  }

  static std::string cors_headers(const ReqRef& r) {
    if (r.origin.empty()) return {};
    return "access-control-allow-origin: " + r.origin + "\r\naccess-control-allow-credentials: true\r\nvary: Origin\r\n";
  }

  static std::string build_response(int code, const std::string& body, const std::string& ctype,
                                    const std::string& extra, bool keep_alive) {
    std::string r;
    r.reserve(body.size() + 160 + extra.size());
    char line[96];
    snprintf(line, sizeof line, "HTTP/1.1 %d %s\r\n", code, reason(code));
    r += line;
    r += "server: mls-native\r\ncontent-type: ";
    r += ctype;
    r += "\r\ncontent-length: ";
    r += std::to_string(body.size());
    r += "\r\n";
    if (!keep_alive) r += "connection: close\r\n";
    r += extra;
    r += "\r\n";
    r += body;
    return r;
  }

  void count(int code) {
    std::lock_guard<std::mutex> g(cmu_);
    code_counts_[code]++;
  }

  // Thread-safe: hand a response to the I/O thread that owns the connection.
  void reply(const ReqRef& ref, int code, const std::string& body, const std::string& ctype = "application/json",
             const std::string& extra = std::string()) {
    count(code);
    if (ref.thread < 0 || ref.thread >= (int)threads_.size()) return;
    IoThread& t = *threads_[ref.thread];
    Outgoing o{ref.conn, build_response(code, body, ctype, cors_headers(ref) + extra, ref.keep_alive),
               !ref.keep_alive};
    bool wake;
    {
      std::lock_guard<std::mutex> g(t.mu);
      wake = t.outbox.empty();
      t.outbox.push_back(std::move(o));
    }
    if (wake) {
      uint64_t one = 1;
      (void)!write(t.efd, &one, sizeof one);
    }
  }

  // ---- I/O thread --------------------------------------------------------------------------
  void io_loop(IoThread& t) {
    std::vector<epoll_event> evs(256);
    while (running_) {
      int n = epoll_wait(t.ep, evs.data(), (int)evs.size(), 200);
      if (n < 0) {
        if (errno == EINTR) continue;
        break;
      }
      for (int i = 0; i < n; ++i) {
        const uint64_t key = evs[i].data.u64;
        if (key == 0) {
          accept_all(t);
        } else if (key == 1) {
          uint64_t v;
          while (read(t.efd, &v, sizeof v) > 0) {
          }
          drain_outbox(t);
        } else {
          auto it = t.conns.find(key);
          if (it == t.conns.end()) continue;
          Conn& c = *it->second;
          const uint32_t e = evs[i].events;
          bool alive = true;
          if (e & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) alive = on_readable(t, c);
          if (alive && (e & EPOLLOUT)) alive = flush(c);
          if (!alive) close_conn(t, key);
        }
      }
    }
  }

  void accept_all(IoThread& t) {
    for (;;) {
      int fd = accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;  // EAGAIN (drained) or a transient error
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      auto c = std::make_unique<Conn>();
      c->fd = fd;
      c->id = next_conn_.fetch_add(1);
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
      ev.data.u64 = c->id;
      if (epoll_ctl(t.ep, EPOLL_CTL_ADD, fd, &ev) != 0) {
        close(fd);
        continue;
      }
      n_conns_++;
      t.conns.emplace(c->id, std::move(c));
    }
  }

  void close_conn(IoThread& t, uint64_t id) {
    auto it = t.conns.find(id);
    if (it == t.conns.end()) return;
    close(it->second->fd);  // also drops it from the epoll set
    t.conns.erase(it);
    n_conns_--;
  }

  void drain_outbox(IoThread& t) {
    std::vector<Outgoing> q;
    {
      std::lock_guard<std::mutex> g(t.mu);
      q.swap(t.outbox);
    }
    for (auto& o : q) {
      auto it = t.conns.find(o.conn);
      if (it == t.conns.end()) continue;  // the client went away
      Conn& c = *it->second;
      c.out.append(o.bytes.data(), o.bytes.size());
      c.waiting = false;
      c.close_after = c.close_after || o.close;
      bool alive = !c.close_after ? process(t, c) : flush(c);  // serve pipelined requests
      if (alive && c.peer_eof && !c.waiting && c.out.size() == 0) alive = false;
      if (!alive) close_conn(t, o.conn);
    }
  }

  // false -> close the connection
  bool flush(Conn& c) {
    while (c.out.size()) {
      ssize_t w = send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) return true;  // EPOLLOUT (edge) resumes
        if (errno == EINTR) continue;
        return false;
      }
      c.out.consume((size_t)w);
    }
    return !c.close_after;
  }

  bool on_readable(IoThread& t, Conn& c) {
    for (;;) {
      c.in.reserve_tail(64 * 1024);
      ssize_t r = recv(c.fd, c.in.p.get() + c.in.end, c.in.cap - c.in.end, 0);
      if (r > 0) {
        c.in.end += (size_t)r;
        if (c.in.size() > (size_t)cfg_.max_upload + 2 * MAX_HEAD) return false;  // runaway pipelining
        continue;
      }
      if (r == 0) {
        c.peer_eof = true;
        break;
      }
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      return false;
    }
    bool alive = process(t, c);
    // half-closed client: finish the outstanding response, then close
    if (alive && c.peer_eof && !c.waiting && c.out.size() == 0) return false;
    return alive;
  }

  static bool parse_head(std::string_view s, Head& h) {
    const size_t end = s.find("\r\n\r\n");
    if (end == std::string_view::npos) return false;
    h.head_len = end + 4;
    const size_t le = s.find("\r\n");
    std::string_view line = s.substr(0, le);
    const size_t sp1 = line.find(' '), sp2 = line.rfind(' ');
    if (sp1 == std::string_view::npos || sp2 == sp1) return true;  // method stays empty -> 400
    h.method = line.substr(0, sp1);
    h.target = line.substr(sp1 + 1, sp2 - sp1 - 1);
    h.http10 = line.substr(sp2 + 1) == "HTTP/1.0";
    const size_t q = h.target.find('?');
    h.path = h.target.substr(0, q);
    h.query = q == std::string_view::npos ? std::string_view() : h.target.substr(q + 1);
    size_t pos = le + 2;
    while (pos < end) {
      size_t e = s.find("\r\n", pos);
      std::string_view hl = s.substr(pos, e - pos);
      pos = e + 2;
      size_t colon = hl.find(':');
      if (colon == std::string_view::npos) continue;
      std::string_view k = trim(hl.substr(0, colon)), v = trim(hl.substr(colon + 1));
      if (ieq(k, "content-length")) {
        long long n = v.empty() ? -2 : 0;
        for (char ch : v) {
          if (ch < '0' || ch > '9' || n > (1LL << 40)) {
            n = -2;
            break;
          }
          n = n * 10 + (ch - '0');
        }
        h.content_length = n;
      } else if (ieq(k, "content-type")) {
        h.content_type = v;
      } else if (ieq(k, "origin")) {
        h.origin = v;
      } else if (ieq(k, "connection")) {
        h.connection = v;
      } else if (ieq(k, "expect")) {
        h.expect = v;
      } else if (ieq(k, "transfer-encoding")) {
        h.transfer_encoding = v;
      } else if (ieq(k, "access-control-request-method")) {
        h.acr_method = v;
      } else if (ieq(k, "access-control-request-headers")) {
        h.acr_headers = v;
      }
    }
    return true;
  }

  bool origin_allowed(std::string_view o) const {
    for (auto& a : cfg_.cors_origins)
      if (a == "*" || a == o) return true;
    return false;
  }

  // Parse and serve every complete request buffered on `c`, one outstanding at a time.
  bool process(IoThread& t, Conn& c) {
    while (!c.waiting && !c.close_after && c.in.size() > 0) {
      std::string_view s(c.in.data(), c.in.size());
      Head h;
      if (!parse_head(s, h)) {
        if (c.in.size() > MAX_HEAD) immediate(c, 431, failure_body("Request headers too large."), false);
        break;  // else: need more bytes
      }
      if (h.head_len > MAX_HEAD) {
        immediate(c, 431, failure_body("Request headers too large."), false);
        break;
      }
      if (h.method.empty()) {
        immediate(c, 400, failure_body("Malformed request line."), false);
        break;
      }
      if (!h.transfer_encoding.empty() && !ieq(h.transfer_encoding, "identity")) {
        immediate(c, 411, failure_body("Chunked request bodies are not supported; send Content-Length."), false);
        break;
      }
      if (h.content_length == -2) {
        immediate(c, 400, failure_body("Invalid Content-Length."), false);
        break;
      }
      const size_t blen = h.content_length > 0 ? (size_t)h.content_length : 0;
      if ((long long)blen > cfg_.max_upload) {
        immediate(c, 413, failure_body("Upload too large."), false);
        break;
      }
      if (c.in.size() < h.head_len + blen) {
        if (!c.sent_continue && istarts(h.expect, "100-continue")) {
          static const char kCont[] = "HTTP/1.1 100 Continue\r\n\r\n";
          c.out.append(kCont, sizeof kCont - 1);
          c.sent_continue = true;
        }
        break;  // body incomplete
      }
      c.sent_continue = false;
      ReqRef ref;
      ref.thread = t.idx;
      ref.conn = c.id;
      ref.t0 = Clock::now();
      ref.keep_alive = h.http10 ? istarts(h.connection, "keep-alive") : !ieq(h.connection, "close");
      if (!h.origin.empty() && origin_allowed(h.origin)) ref.origin = std::string(h.origin);
      n_requests_++;
      handle(c, h, std::string_view(c.in.data() + h.head_len, blen), std::move(ref));
      c.in.consume(h.head_len + blen);
    }
    return flush(c);
  }

  // A response produced on the I/O thread itself.
  void immediate(Conn& c, int code, const std::string& body, bool keep_alive, const std::string& extra = {},
                 const char* ctype = "application/json") {
    count(code);
    std::string r = build_response(code, body, ctype, extra, keep_alive);
    c.out.append(r.data(), r.size());
    if (!keep_alive) {
      c.close_after = true;
      c.in.consume(c.in.size());
    }
  }

  void to_python(Conn& c, const Head& h, std::string_view body, ReqRef ref) {
    PyRequest r;
    r.method = std::string(h.method);
    r.path = std::string(h.path);
    r.query = std::string(h.query);
    std::string_view s(c.in.data(), h.head_len - 2);  // header block incl. the last line's CRLF
    size_t pos = s.find("\r\n") + 2;
    while (pos < s.size()) {
      size_t e = s.find("\r\n", pos);
      if (e == std::string_view::npos) break;
      std::string_view hl = s.substr(pos, e - pos);
      size_t colon = hl.find(':');
      if (colon != std::string_view::npos) {
        std::string k(trim(hl.substr(0, colon)));
        std::transform(k.begin(), k.end(), k.begin(), [](unsigned char ch) { return (char)tolower(ch); });
        r.headers.emplace_back(std::move(k), std::string(trim(hl.substr(colon + 1))));
      }
      pos = e + 2;
    }
    r.body.assign(body.data(), body.size());
    r.token = new_token(std::move(ref));
    n_python_++;
    c.waiting = true;
    {
      std::lock_guard<std::mutex> g(qmu_);
      req_q_.push_back(std::move(r));
    }
    rcv_.notify_one();
  }

  void handle(Conn& c, const Head& h, std::string_view body, ReqRef ref) {
    const std::string cors = cors_headers(ref);
    // CORS preflight (starlette CORSMiddleware semantics for an explicit origin list)
    if (h.method == "OPTIONS" && !h.origin.empty() && !h.acr_method.empty()) {
      if (!ref.origin.empty()) {
        std::string extra = "access-control-allow-origin: " + ref.origin +
                            "\r\naccess-control-allow-credentials: true\r\n"
                            "access-control-allow-methods: DELETE, GET, HEAD, OPTIONS, PATCH, POST, PUT\r\n"
                            "access-control-max-age: 600\r\nvary: Origin\r\n";
        if (!h.acr_headers.empty()) extra += "access-control-allow-headers: " + std::string(h.acr_headers) + "\r\n";
        immediate(c, 200, "OK", ref.keep_alive, extra, "text/plain; charset=utf-8");
      } else {
        immediate(c, 400, "Disallowed CORS origin", ref.keep_alive, "vary: Origin\r\n", "text/plain; charset=utf-8");
      }
      return;
    }
    if (h.path == "/" && h.method == "GET") {
      immediate(c, 200, ROOT_BODY, ref.keep_alive, cors);
      return;
    }
    if (h.path == "/status" && h.method == "GET") {
      bool ready;
      std::string err;
      {
        std::lock_guard<std::mutex> g(state_mu_);
        ready = ready_;
        err = init_error_;
      }
      if (ready) {
        immediate(c, 200, READY_BODY, ref.keep_alive, cors);
      } else if (!err.empty()) {
        std::string b = "{\"status\":\"failure\",\"detail\":\"Model is not ready to receive predictions.\",\"error\":";
        json_escape(b, err);
        b += "}";
        immediate(c, 503, b, ref.keep_alive, cors);
      } else {
        immediate(c, 503, NOT_READY_BODY, ref.keep_alive, cors);
      }
      return;
    }
    if (!(h.path == "/predict" && h.method == "POST")) {
      to_python(c, h, body, std::move(ref));  // /health, /metrics, /info, 404 / 405 ...
      return;
    }
    // ---- POST /predict ----
    std::string_view payload, pctype;
    bool found = false;
    bool legacy = h.query.find("filename=") != std::string_view::npos;
    if (istarts(h.content_type, "multipart/form-data")) {
      std::vector<Part> parts;
      if (!parse_multipart(body, header_param(h.content_type, "boundary"), parts)) {
        immediate(c, 400, failure_body("Malformed upload: bad multipart framing"), ref.keep_alive, cors);
        return;
      }
      for (auto& p : parts) {
        if (p.name == cfg_.form_field) {
          payload = p.data;
          pctype = p.content_type;
          found = true;
          break;
        }
        if (p.name == "filename") legacy = true;
      }
    } else if (istarts(h.content_type, "application/octet-stream") || istarts(h.content_type, "application/x-rgb8")) {
      payload = body;
      pctype = h.content_type;
      found = true;
    } else if (istarts(h.content_type, "application/json") ||
               istarts(h.content_type, "application/x-www-form-urlencoded")) {
      to_python(c, h, body, std::move(ref));  // text fields / legacy filename: the Python handler's job
      return;
    }
    if (!found) {
      if (legacy) {
        to_python(c, h, body, std::move(ref));  // old-rev ?filename= shared-volume flow
        return;
      }
      std::string b = "{\"detail\":[{\"type\":\"missing\",\"loc\":[\"body\",";
      json_escape(b, cfg_.form_field);
      b += "],\"msg\":\"Field required\",\"input\":null}]}";
      immediate(c, 422, b, ref.keep_alive, cors);
      return;
    }
    bool ready;
    {
      std::lock_guard<std::mutex> g(state_mu_);
      ready = ready_;
    }
    if (!ready) {
      immediate(c, 503, NOT_READY_BODY, ref.keep_alive, cors);
      return;
    }
    if (cfg_.image_container) {
      Pending p;
      p.body.assign(mlsjpeg::CONTAINER_BYTES, '\0');
      uint8_t* dst = reinterpret_cast<uint8_t*>(&p.body[0]);
      bool ok = false;
      if (payload.size() == mlsjpeg::PAYLOAD_BYTES && raw_content_type(pctype)) {
        mlsjpeg::raw_container(reinterpret_cast<const uint8_t*>(payload.data()), dst);
        ok = true;
      } else if (payload.size() > 2 && (uint8_t)payload[0] == 0xFF && (uint8_t)payload[1] == 0xD8) {
        ok = mlsjpeg::jpeg_to_container(reinterpret_cast<const uint8_t*>(payload.data()), payload.size(), dst);
        if (ok) n_jpeg_native_++;
      }
      if (ok) {
        p.ref = std::move(ref);
        p.off = 0;
        c.waiting = true;
        enqueue_sample(std::move(p));
        return;
      }
      // not raw, not a baseline JPEG this decoder takes: the Python (PIL) decode threads below
    } else if (cfg_.raw_samples && cfg_.sample_bytes > 0 && (long long)payload.size() == cfg_.sample_bytes &&
        raw_content_type(pctype)) {
      Pending p;
      p.ref = std::move(ref);
      p.off = (size_t)(payload.data() - body.data());
      p.body.assign(body.data(), body.size());
      c.waiting = true;
      enqueue_sample(std::move(p));
      return;
    }
    if (cfg_.text_hash.vocab > 0) {
      std::vector<int32_t> ids;
      if (hash_tokenize(payload, cfg_.text_hash, ids)) {
        const int S = cfg_.text_hash.seq;
        std::vector<int32_t> row(2 * S + 1, 0);
        std::copy(ids.begin(), ids.end(), row.begin());
        row[2 * S] = (int32_t)ids.size();
        Pending p;
        p.ref = std::move(ref);
        p.body.assign(reinterpret_cast<const char*>(row.data()), row.size() * sizeof(int32_t));
        c.waiting = true;
        n_text_hash_++;
        enqueue_sample(std::move(p));
        return;
      }
    }
    if (!cfg_.python_decode) {
      immediate(c, 415, failure_body("Only raw samples of the model's input size are accepted."), ref.keep_alive, cors);
      return;
    }
    DecodeItem d;
    d.data.assign(payload.data(), payload.size());
    d.ctype = std::string(pctype);
    d.token = new_token(std::move(ref));
    n_decode_++;
    c.waiting = true;
    {
      std::lock_guard<std::mutex> g(qmu_);
      decode_q_.push_back(std::move(d));
    }
    dcv_.notify_one();
  }
};

py::bytes as_bytes(const std::string& s) { return py::bytes(s.data(), s.size()); }

}  // namespace

PYBIND11_MODULE(_httpfront, m) {
  m.doc() = "Native HTTP/1.1 front end: epoll I/O threads, multipart parsing, C++ dynamic batching";
  m.def("jpeg_container",
        [](py::bytes data) -> py::object {
          std::string in = data;
          std::string out(mlsjpeg::CONTAINER_BYTES, '\0');
          std::string why;
          bool ok;
          {
            py::gil_scoped_release rel;
            ok = mlsjpeg::jpeg_to_container(reinterpret_cast<const uint8_t*>(in.data()), in.size(),
                                            reinterpret_cast<uint8_t*>(&out[0]), &why);
          }
          if (!ok) return py::str(why);
          return py::bytes(out);
        },
        "JPEG bytes -> GPU image container (bytes), or the reason (str) it is not handled");
  m.def("raw_container",
        [](py::bytes rgb) -> py::bytes {
          std::string in = rgb;
          if (in.size() != mlsjpeg::PAYLOAD_BYTES) throw std::invalid_argument("raw image must be 224 x 224 x 3 bytes");
          std::string out(mlsjpeg::CONTAINER_BYTES, '\0');
          mlsjpeg::raw_container(reinterpret_cast<const uint8_t*>(in.data()), reinterpret_cast<uint8_t*>(&out[0]));
          return py::bytes(out);
        });
  m.attr("CONTAINER_BYTES") = (long long)mlsjpeg::CONTAINER_BYTES;
  m.def("hash_tokenize",
        [](std::string text, int vocab, int max_len, int seq) -> py::object {
          std::vector<int32_t> ids;
          if (!hash_tokenize(text, TextHash{vocab, max_len, seq, 101, 102}, ids)) return py::none();
          return py::cast(ids);
        },
        "C++ hash tokenizer of the bert plugin (None for non-ASCII text)", py::arg("text"), py::arg("vocab"),
        py::arg("max_len"), py::arg("seq"));
  py::class_<Server>(m, "Server")
      .def(py::init([](std::string host, int port, int listen_fd, int io_threads, long long sample_bytes,
                       int max_batch, int max_wait_us, int max_queue, long long max_upload, std::string form_field,
                       std::vector<std::string> cors_origins, double request_timeout_s, bool python_decode,
                       bool raw_samples, std::vector<int> text_hash, bool image_container) {
             Server::Config c;
             c.host = std::move(host);
             c.port = port;
             c.listen_fd = listen_fd;
             c.io_threads = io_threads;
             c.sample_bytes = sample_bytes;
             c.max_batch = max_batch;
             c.max_wait_us = max_wait_us;
             c.max_queue = max_queue;
             c.max_upload = max_upload;
             c.form_field = std::move(form_field);
             c.cors_origins = std::move(cors_origins);
             c.request_timeout_s = request_timeout_s;
             c.python_decode = python_decode;
             c.raw_samples = raw_samples;
             c.image_container = image_container;
             if (image_container && c.sample_bytes != (long long)mlsjpeg::CONTAINER_BYTES)
               throw std::invalid_argument("image_container needs sample_bytes == CONTAINER_BYTES");
             if (text_hash.size() == 5) {  // vocab, max_len, seq, cls, sep
               c.text_hash = TextHash{text_hash[0], text_hash[1], text_hash[2], text_hash[3], text_hash[4]};
               if (c.text_hash.vocab <= 1000 || c.text_hash.seq <= 0 || c.text_hash.max_len < 2 ||
                   c.sample_bytes != (long long)(2 * c.text_hash.seq + 1) * 4)
                 throw std::invalid_argument("text_hash does not match sample_bytes");
             }
             return std::make_unique<Server>(std::move(c));
           }),
           py::arg("host") = "0.0.0.0", py::arg("port") = 0, py::arg("listen_fd") = -1, py::arg("io_threads") = 4,
           py::arg("sample_bytes") = 0, py::arg("max_batch") = 32, py::arg("max_wait_us") = 2000,
           py::arg("max_queue") = 4096, py::arg("max_upload") = 32 << 20, py::arg("form_field") = "image_file",
           py::arg("cors_origins") = std::vector<std::string>{}, py::arg("request_timeout_s") = 30.0,
           py::arg("python_decode") = true, py::arg("raw_samples") = true,
           py::arg("text_hash") = std::vector<int>{}, py::arg("image_container") = false)
      .def("start", &Server::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Server::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Server::port)
      .def("set_ready", &Server::set_ready, py::arg("ready"), py::arg("error") = "")
      .def("set_labels", &Server::set_labels)
      .def(
          "next_batch",
          [](Server& s, py::buffer dst, int cap, int timeout_ms) -> py::object {
            py::buffer_info bi = dst.request(true);
            char* p = static_cast<char*>(bi.ptr);
            const size_t nbytes = (size_t)bi.size * (size_t)bi.itemsize;
            std::pair<uint64_t, int> r;
            {
              py::gil_scoped_release nogil;
              r = s.next_batch(p, nbytes, cap, timeout_ms);
            }
            if (r.second == 0) return py::none();
            return py::make_tuple(r.first, r.second);
          },
          py::arg("dst"), py::arg("cap"), py::arg("timeout_ms") = 200)
      .def(
          "complete_topk",
          [](Server& s, uint64_t id, py::array_t<float, py::array::c_style | py::array::forcecast> vals,
             py::array_t<int32_t, py::array::c_style | py::array::forcecast> idx) {
            if (vals.ndim() != 2 || idx.ndim() != 2 || vals.shape(0) != idx.shape(0) || vals.shape(1) != idx.shape(1))
              throw std::runtime_error("complete_topk: vals / idx must both be [n, k]");
            const float* v = vals.data();
            const int32_t* i = idx.data();
            const int n = (int)vals.shape(0), k = (int)vals.shape(1);
            py::gil_scoped_release nogil;
            s.complete_topk(id, v, i, n, k);
          },
          py::arg("batch_id"), py::arg("vals"), py::arg("idx"))
      .def("complete_json", &Server::complete_json, py::call_guard<py::gil_scoped_release>())
      .def("fail_batch", &Server::fail_batch, py::call_guard<py::gil_scoped_release>())
      .def(
          "next_decode",
          [](Server& s, int timeout_ms) -> py::object {
            DecodeItem d;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.next_decode(timeout_ms, d);
            }
            if (!ok) return py::none();
            return py::make_tuple(d.token, as_bytes(d.data), d.ctype);
          },
          py::arg("timeout_ms") = 200)
      .def(
          "submit_sample",
          [](Server& s, uint64_t token, py::buffer sample) {
            py::buffer_info bi = sample.request();
            const size_t n = (size_t)bi.size * (size_t)bi.itemsize;
            const char* p = static_cast<const char*>(bi.ptr);
            py::gil_scoped_release nogil;
            return s.submit_sample(token, p, n);
          },
          py::arg("token"), py::arg("sample"))
      .def(
          "next_request",
          [](Server& s, int timeout_ms) -> py::object {
            PyRequest r;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.next_request(timeout_ms, r);
            }
            if (!ok) return py::none();
            py::dict h;
            for (auto& kv : r.headers) h[py::str(kv.first)] = py::str(kv.second);
            return py::make_tuple(r.token, r.method, r.path, r.query, h, as_bytes(r.body));
          },
          py::arg("timeout_ms") = 200)
      .def(
          "respond",
          [](Server& s, uint64_t token, int code, py::bytes body, std::string ctype,
             std::vector<std::pair<std::string, std::string>> headers) {
            std::string b = body;
            py::gil_scoped_release nogil;
            return s.respond(token, code, b, ctype, headers);
          },
          py::arg("token"), py::arg("status"), py::arg("body"), py::arg("content_type") = "application/json",
          py::arg("headers") = std::vector<std::pair<std::string, std::string>>{})
      .def("stats", &Server::stats);
}
