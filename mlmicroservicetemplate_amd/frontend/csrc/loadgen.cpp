// mls_loadgen: closed-loop HTTP/1.1 keep-alive load generator for POST /predict.
//
// The Python/aiohttp generator (tools/loadgen.py) tops out at a few thousand requests/s per
// process, below what the native front end serves; this one keeps `--conns` connections busy
// from `--threads` epoll threads, each connection sending its next request as soon as the
// previous response is complete.  Payload: a random raw RGB8 sample of `--bytes` bytes, sent as
// multipart field `--field` (default image_file, application/octet-stream) or, with --raw, as
// the whole application/octet-stream body.  Prints one JSON line (requests/s, latency
// percentiles over the measured window, status-code counts).
//
// usage: mls_loadgen --port P [--host 127.0.0.1] [--path /predict] [--conns 64] [--threads 4]
//                    [--duration 10] [--warmup 2] [--bytes 150528] [--field image_file] [--raw]
//                    [--file upload.jpg --ctype image/jpeg]   (a real file instead of random bytes)
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

namespace {

struct Opts {
  std::string host = "127.0.0.1";
  int port = 5005;
  std::string path = "/predict";
  int conns = 64, threads = 4;
  double duration = 10, warmup = 2;
  long bytes = 224 * 224 * 3;
  std::string field = "image_file";
  bool raw = false;
  std::string file;                            // send this file's bytes instead of random ones
  std::string ctype = "application/octet-stream";  // the upload part's content type
};

struct ThreadStats {
  std::vector<float> lat_ms;
  std::map<int, long> codes;
  long ok = 0, errors = 0, reconnects = 0;
};

struct Conn {
  int fd = -1;
  size_t sent = 0;
  std::string in;
  Clock::time_point t0;
  bool connected = false;
};

int open_conn(const Opts& o) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)o.port);
  inet_pton(AF_INET, o.host.c_str(), &a.sin_addr);
  if (connect(fd, (sockaddr*)&a, sizeof a) != 0 && errno != EINPROGRESS) {
    close(fd);
    return -1;
  }
  return fd;
}

// A complete response in `in`?  Returns its total length (0 if incomplete, -1 if malformed)
// and its status code.
long response_len(const std::string& in, int& status) {
  size_t he = in.find("\r\n\r\n");
  if (he == std::string::npos) return 0;
  if (in.compare(0, 5, "HTTP/") != 0) return -1;
  size_t sp = in.find(' ');
  status = atoi(in.c_str() + sp + 1);
  if (status == 100) return (long)(he + 4);  // interim response: skip it
  long clen = 0;
  size_t pos = in.find("\r\n") + 2;
  while (pos < he) {
    size_t e = in.find("\r\n", pos);
    if (e - pos > 15 && strncasecmp(in.c_str() + pos, "content-length:", 15) == 0) clen = atol(in.c_str() + pos + 15);
    pos = e + 2;
  }
  long total = (long)(he + 4) + clen;
  return (long)in.size() >= total ? total : 0;
}

void worker(const Opts& o, const std::string& req, int nconn, Clock::time_point t_measure, Clock::time_point t_end,
            ThreadStats& st) {
  int ep = epoll_create1(EPOLL_CLOEXEC);
  std::vector<Conn> cs(nconn);
  auto arm = [&](int i) {
    Conn& c = cs[i];
    c.fd = open_conn(o);
    c.sent = 0;
    c.in.clear();
    c.t0 = Clock::now();
    if (c.fd < 0) return;
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLOUT | EPOLLET;
    ev.data.u32 = (uint32_t)i;
    epoll_ctl(ep, EPOLL_CTL_ADD, c.fd, &ev);
  };
  auto reset = [&](int i) {
    if (cs[i].fd >= 0) close(cs[i].fd);
    st.reconnects++;
    arm(i);
  };
  for (int i = 0; i < nconn; ++i) arm(i);
  std::vector<epoll_event> evs(256);
  char buf[65536];
  while (Clock::now() < t_end) {
    int n = epoll_wait(ep, evs.data(), (int)evs.size(), 50);
    for (int k = 0; k < n; ++k) {
      int i = (int)evs[k].data.u32;
      Conn& c = cs[i];
      if (c.fd < 0) continue;
      bool dead = (evs[k].events & (EPOLLERR | EPOLLHUP)) != 0;
      // send what is left of the current request
      while (!dead && c.sent < req.size()) {
        ssize_t w = send(c.fd, req.data() + c.sent, req.size() - c.sent, MSG_NOSIGNAL);
        if (w < 0) {
          if (errno != EAGAIN && errno != EWOULDBLOCK) dead = true;
          break;
        }
        c.sent += (size_t)w;
      }
      // read responses
      while (!dead) {
        ssize_t r = recv(c.fd, buf, sizeof buf, 0);
        if (r > 0) {
          c.in.append(buf, (size_t)r);
          continue;
        }
        if (r == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) dead = true;
        break;
      }
      for (;;) {
        int status = 0;
        long len = dead && c.in.empty() ? 0 : response_len(c.in, status);
        if (len < 0) {
          dead = true;
          break;
        }
        if (len == 0) break;
        c.in.erase(0, (size_t)len);
        if (status == 100) continue;
        auto now = Clock::now();
        if (c.t0 >= t_measure) {
          st.codes[status]++;
          if (status == 200) {
            st.ok++;
            st.lat_ms.push_back(std::chrono::duration<float, std::milli>(now - c.t0).count());
          } else {
            st.errors++;
          }
        }
        // next request on the same connection
        c.t0 = now;
        c.sent = 0;
        while (c.sent < req.size()) {
          ssize_t w = send(c.fd, req.data() + c.sent, req.size() - c.sent, MSG_NOSIGNAL);
          if (w < 0) {
            if (errno != EAGAIN && errno != EWOULDBLOCK) dead = true;
            break;
          }
          c.sent += (size_t)w;
        }
        break;
      }
      if (dead) {
        if (c.t0 >= t_measure) st.errors++;
        reset(i);
      }
    }
  }
  for (auto& c : cs)
    if (c.fd >= 0) close(c.fd);
  close(ep);
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") o.host = next();
    else if (a == "--port") o.port = atoi(next());
    else if (a == "--path") o.path = next();
    else if (a == "--conns") o.conns = atoi(next());
    else if (a == "--threads") o.threads = atoi(next());
    else if (a == "--duration") o.duration = atof(next());
    else if (a == "--warmup") o.warmup = atof(next());
    else if (a == "--bytes") o.bytes = atol(next());
    else if (a == "--field") o.field = next();
    else if (a == "--raw") o.raw = true;
    else if (a == "--file") o.file = next();
    else if (a == "--ctype") o.ctype = next();
    else {
      fprintf(stderr, "unknown option %s\n", a.c_str());
      return 2;
    }
  }
  o.threads = std::max(1, std::min(o.threads, o.conns));
  std::string payload;
  if (!o.file.empty()) {
    FILE* f = fopen(o.file.c_str(), "rb");
    if (!f) {
      fprintf(stderr, "cannot open %s\n", o.file.c_str());
      return 2;
    }
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) payload.append(buf, n);
    fclose(f);
    o.bytes = (long)payload.size();
  } else {
    std::mt19937 rng(1234);
    payload.assign((size_t)o.bytes, '\0');
    for (auto& ch : payload) ch = (char)(rng() & 0xff);
  }
  std::string body, ctype;
  if (o.raw) {
    body = payload;
    ctype = o.ctype;
  } else {
    const std::string bnd = "mlsloadgenboundary7d1f";
    body = "--" + bnd + "\r\nContent-Disposition: form-data; name=\"" + o.field +
           "\"; filename=\"upload\"\r\nContent-Type: " + o.ctype + "\r\n\r\n" + payload + "\r\n--" + bnd +
           "--\r\n";
    ctype = "multipart/form-data; boundary=" + bnd;
  }
  std::string req = "POST " + o.path + " HTTP/1.1\r\nHost: " + o.host + "\r\nContent-Type: " + ctype +
                    "\r\nContent-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  auto t_start = Clock::now();
  auto t_measure = t_start + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(o.warmup));
  auto t_end = t_measure + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(o.duration));
  std::vector<ThreadStats> stats(o.threads);
  std::vector<std::thread> ths;
  for (int t = 0; t < o.threads; ++t) {
    int nconn = o.conns / o.threads + (t < o.conns % o.threads ? 1 : 0);
    ths.emplace_back(worker, std::cref(o), std::cref(req), nconn, t_measure, t_end, std::ref(stats[t]));
  }
  for (auto& th : ths) th.join();
  std::vector<float> lat;
  std::map<int, long> codes;
  long ok = 0, errors = 0, reconnects = 0;
  for (auto& s : stats) {
    lat.insert(lat.end(), s.lat_ms.begin(), s.lat_ms.end());
    for (auto& kv : s.codes) codes[kv.first] += kv.second;
    ok += s.ok;
    errors += s.errors;
    reconnects += s.reconnects;
  }
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double p) -> double {
    if (lat.empty()) return 0.0;
    size_t i = std::min(lat.size() - 1, (size_t)(p * (double)(lat.size() - 1) + 0.5));
    return lat[i];
  };
  printf("{\"metric\": \"http requests/sec + latency\", \"client\": \"mls_loadgen\", \"conns\": %d, \"threads\": %d, "
         "\"payload_bytes\": %ld, \"multipart\": %s, \"duration_s\": %.2f, \"requests_per_s\": %.1f, "
         "\"p50_ms\": %.3f, \"p90_ms\": %.3f, \"p99_ms\": %.3f, \"ok\": %ld, \"errors\": %ld, \"reconnects\": %ld, "
         "\"status_codes\": {",
         o.conns, o.threads, o.bytes, o.raw ? "false" : "true", o.duration, ok / o.duration, pct(0.5), pct(0.9),
         pct(0.99), ok, errors, reconnects);
  bool first = true;
  for (auto& kv : codes) {
    printf("%s\"%d\": %ld", first ? "" : ", ", kv.first, kv.second);
    first = false;
  }
  printf("}}\n");
  return 0;
}
