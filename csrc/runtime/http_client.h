// Closed-loop HTTP/1.1 client core (keep-alive, one request in flight per connection, responses
// framed by Content-Length).  Shared by the standalone load generator (csrc/tools/loadgen.cpp) and
// the _rt.http_load binding that bench.py uses to time single requests without the Python client's
// own ~30 us per round trip in the measurement.
#pragma once
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace rtc {

struct LoadResult {
  double seconds = 0;
  long long requests = 0, errors = 0, bytes = 0;
  // per request kind: responses by status code (http_load_mixed)
  std::vector<std::vector<std::pair<int, long long>>> status_by_kind;
  std::vector<float> lat_us;   // sorted per-request latencies
  std::vector<std::pair<float, float>> p50_p99_by_kind;   // http_load_mixed: per kind (us)
  double pct(double p) const {
    return lat_us.empty() ? 0.0 : (double)lat_us[std::min(lat_us.size() - 1, (size_t)(p * lat_us.size()))];
  }
};

inline std::string post_request(const std::string& path, const std::string& body) {
  return "POST " + path + " HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: application/json\r\n" +
         "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
}

// nconn connections over nthreads epoll loops; runs until `seconds` elapse or `max_requests`
// responses (0 = unlimited) have arrived.  Every new request takes the next of `reqs` (whole HTTP
// requests, cycled by a shared counter).  The first `warmup` responses per connection are not
// recorded.
inline LoadResult http_load_multi(int port, int nconn, double seconds, const std::vector<std::string>& reqs,
                                  int nthreads, long long max_requests = 0, int warmup = 0) {
  using Clock = std::chrono::steady_clock;
  struct C {
    int fd = -1;
    std::string in;
    Clock::time_point t0;
    int seen = 0;
  };
  nthreads = std::max(1, std::min(nthreads, std::max(1, nconn)));
  std::atomic<long long> total{0}, errors{0}, bytes{0}, next{0};
  auto send_next = [&](int fd) {
    const std::string& req = reqs[(size_t)(next.fetch_add(1, std::memory_order_relaxed) % (long long)reqs.size())];
    size_t off = 0;
    while (off < req.size()) {
      const ssize_t w = write(fd, req.data() + off, req.size() - off);
      if (w <= 0) { errors++; return; }
      off += (size_t)w;
    }
  };
  std::vector<std::vector<float>> lat(nthreads);
  const auto t_end = Clock::now() + std::chrono::microseconds((long long)(seconds * 1e6));
  auto done = [&](Clock::time_point now) {
    return now >= t_end || (max_requests > 0 && total.load(std::memory_order_relaxed) >= max_requests);
  };
  auto worker = [&](int tid) {
    const int mine = nconn / nthreads + (tid < nconn % nthreads);
    const int ep = epoll_create1(0);
    std::vector<C> cs(mine);
    for (int i = 0; i < mine; ++i) {
      int fd = socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)port);
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      if (connect(fd, (sockaddr*)&a, sizeof a) != 0) { errors++; close(fd); continue; }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      cs[i].fd = fd;
      epoll_event e{};
      e.events = EPOLLIN;
      e.data.u32 = (uint32_t)i;
      epoll_ctl(ep, EPOLL_CTL_ADD, fd, &e);
      cs[i].t0 = Clock::now();
      send_next(fd);
    }
    std::vector<float>& L = lat[tid];
    epoll_event evs[512];
    std::vector<char> buf(1 << 16);
    bool stop = false;
    while (!stop && !done(Clock::now())) {
      const int n = epoll_wait(ep, evs, 512, 50);
      for (int k = 0; k < n; ++k) {
        C& c = cs[evs[k].data.u32];
        const ssize_t r = read(c.fd, buf.data(), buf.size());
        if (r <= 0) { errors++; stop = true; break; }
        c.in.append(buf.data(), (size_t)r);
        while (true) {
          const size_t h = c.in.find("\r\n\r\n");
          if (h == std::string::npos) break;
          size_t clen = 0;
          size_t cl = c.in.find("content-length:");
          if (cl == std::string::npos || cl > h) cl = c.in.find("Content-Length:");
          if (cl != std::string::npos && cl < h) clen = std::strtoull(c.in.c_str() + cl + 15, nullptr, 10);
          if (c.in.size() < h + 4 + clen) break;
          if (c.in.compare(0, 12, "HTTP/1.1 200") != 0) errors++;
          bytes += (long long)(h + 4 + clen);
          c.in.erase(0, h + 4 + clen);
          const auto now = Clock::now();
          if (c.seen++ >= warmup) {
            L.push_back((float)std::chrono::duration<double, std::micro>(now - c.t0).count());
            total++;
          }
          if (!done(now)) {
            c.t0 = Clock::now();
            send_next(c.fd);
          }
        }
      }
    }
    for (auto& c : cs)
      if (c.fd >= 0) close(c.fd);
    close(ep);
  };
  const auto t0 = Clock::now();
  std::vector<std::thread> th;
  for (int i = 0; i < nthreads; ++i) th.emplace_back(worker, i);
  for (auto& t : th) t.join();
  LoadResult res;
  res.seconds = std::chrono::duration<double>(Clock::now() - t0).count();
  for (auto& v : lat) res.lat_us.insert(res.lat_us.end(), v.begin(), v.end());
  std::sort(res.lat_us.begin(), res.lat_us.end());
  res.requests = total.load();
  res.errors = errors.load();
  res.bytes = bytes.load();
  return res;
}

// Mixed traffic: raw HTTP requests `reqs` (any method) with a kind id each, picked round-robin by
// a shared counter; every response's status code is tallied per kind (contract checks happen in
// the caller).  Responses are framed by Content-Length (none = empty body, e.g. 204).
inline LoadResult http_load_mixed(int port, int nconn, double seconds, const std::vector<std::string>& reqs,
                                  const std::vector<int>& kinds, int nkinds, int nthreads) {
  using Clock = std::chrono::steady_clock;
  struct C {
    int fd = -1;
    std::string in;
    Clock::time_point t0;
    int kind = 0;
  };
  nthreads = std::max(1, std::min(nthreads, std::max(1, nconn)));
  std::atomic<long long> total{0}, errors{0}, bytes{0}, next{0};
  std::vector<std::vector<std::vector<long long>>> counts(nthreads, std::vector<std::vector<long long>>(nkinds, std::vector<long long>(600, 0)));
  std::vector<std::vector<float>> lat(nthreads);
  std::vector<std::vector<std::vector<float>>> lat_k(nthreads, std::vector<std::vector<float>>(nkinds));
  const auto t_end = Clock::now() + std::chrono::microseconds((long long)(seconds * 1e6));
  auto send_next = [&](C& c) {
    const size_t k = (size_t)(next.fetch_add(1, std::memory_order_relaxed) % (long long)reqs.size());
    c.kind = kinds[k];
    const std::string& req = reqs[k];
    size_t off = 0;
    while (off < req.size()) {
      const ssize_t w = write(c.fd, req.data() + off, req.size() - off);
      if (w <= 0) { errors++; return; }
      off += (size_t)w;
    }
  };
  auto worker = [&](int tid) {
    const int mine = nconn / nthreads + (tid < nconn % nthreads);
    const int ep = epoll_create1(0);
    std::vector<C> cs(mine);
    for (int i = 0; i < mine; ++i) {
      int fd = socket(AF_INET, SOCK_STREAM, 0);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)port);
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      if (connect(fd, (sockaddr*)&a, sizeof a) != 0) { errors++; close(fd); continue; }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      cs[i].fd = fd;
      epoll_event e{};
      e.events = EPOLLIN;
      e.data.u32 = (uint32_t)i;
      epoll_ctl(ep, EPOLL_CTL_ADD, fd, &e);
      cs[i].t0 = Clock::now();
      send_next(cs[i]);
    }
    epoll_event evs[512];
    std::vector<char> buf(1 << 16);
    bool stop = false;
    while (!stop && Clock::now() < t_end) {
      const int n = epoll_wait(ep, evs, 512, 50);
      for (int k = 0; k < n; ++k) {
        C& c = cs[evs[k].data.u32];
        const ssize_t r = read(c.fd, buf.data(), buf.size());
        if (r <= 0) { errors++; stop = true; break; }
        c.in.append(buf.data(), (size_t)r);
        while (true) {
          const size_t h = c.in.find("\r\n\r\n");
          if (h == std::string::npos) break;
          size_t clen = 0;
          for (const char* key : {"content-length:", "Content-Length:"}) {
            const size_t cl = c.in.find(key);
            if (cl != std::string::npos && cl < h) { clen = std::strtoull(c.in.c_str() + cl + 15, nullptr, 10); break; }
          }
          if (c.in.size() < h + 4 + clen) break;
          const int code = c.in.size() > 12 ? std::atoi(c.in.c_str() + 9) : 0;
          counts[tid][c.kind][(code >= 0 && code < 600) ? code : 0]++;
          bytes += (long long)(h + 4 + clen);
          c.in.erase(0, h + 4 + clen);
          const auto now = Clock::now();
          const float us = (float)std::chrono::duration<double, std::micro>(now - c.t0).count();
          lat[tid].push_back(us);
          lat_k[tid][c.kind].push_back(us);
          total++;
          if (now < t_end) {
            c.t0 = Clock::now();
            send_next(c);
          }
        }
      }
    }
    for (auto& c : cs)
      if (c.fd >= 0) close(c.fd);
    close(ep);
  };
  const auto t0 = Clock::now();
  std::vector<std::thread> th;
  for (int i = 0; i < nthreads; ++i) th.emplace_back(worker, i);
  for (auto& t : th) t.join();
  LoadResult res;
  res.seconds = std::chrono::duration<double>(Clock::now() - t0).count();
  for (auto& v : lat) res.lat_us.insert(res.lat_us.end(), v.begin(), v.end());
  std::sort(res.lat_us.begin(), res.lat_us.end());
  res.requests = total.load();
  res.errors = errors.load();
  res.bytes = bytes.load();
  res.status_by_kind.resize(nkinds);
  for (int k = 0; k < nkinds; ++k)
    for (int code = 0; code < 600; ++code) {
      long long c = 0;
      for (int t = 0; t < nthreads; ++t) c += counts[t][k][code];
      if (c) res.status_by_kind[k].emplace_back(code, c);
    }
  for (int k = 0; k < nkinds; ++k) {
    std::vector<float> v;
    for (int t = 0; t < nthreads; ++t) v.insert(v.end(), lat_k[t][k].begin(), lat_k[t][k].end());
    std::sort(v.begin(), v.end());
    auto at = [&](double p) { return v.empty() ? 0.f : v[std::min(v.size() - 1, (size_t)(p * v.size()))]; };
    res.p50_p99_by_kind.emplace_back(at(0.5), at(0.99));
  }
  return res;
}

inline LoadResult http_load(int port, int nconn, double seconds, const std::string& path,
                            const std::string& body, int nthreads, long long max_requests = 0,
                            int warmup = 0) {
  return http_load_multi(port, nconn, seconds, {post_request(path, body)}, nthreads, max_requests, warmup);
}

}  // namespace rtc
