// Closed-loop HTTP/1.1 load generator for the prediction endpoints (wrk is not in the image).
//
//   loadgen <port> <connections> <seconds> [path] [body-file|-] [threads]
//
// Each connection keeps one request in flight (keep-alive); responses are parsed by
// Content-Length.  Prints one JSON line: requests/s, latency p50/p90/p99/max (us), errors.
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

struct C {
  int fd;
  std::string in;
  Clock::time_point t0;
  size_t sent = 0;
};

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: loadgen port connections seconds [path] [body-file|-] [threads]\n");
    return 2;
  }
  const int port = std::atoi(argv[1]);
  const int nconn = std::atoi(argv[2]);
  const double secs = std::atof(argv[3]);
  const std::string path = argc > 4 ? argv[4] : "/api/predict_eta";
  std::string body =
      "{\"summary\":{\"distance\":12345},\"pickup_time\":\"2026-10-15T08:30:00\",\"driver_age\":34,"
      "\"weather\":\"Sunny\",\"traffic\":\"Medium\"}";
  if (argc > 5 && std::string(argv[5]) != "-") {
    std::ifstream f(argv[5], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    body = ss.str();
  }
  const int nthreads = argc > 6 ? std::max(1, std::atoi(argv[6])) : 4;
  const std::string req = "POST " + path + " HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: application/json\r\n" +
                          "Content-Length: " + std::to_string(body.size()) + "\r\n\r\n" + body;
  std::atomic<long long> total{0}, errors{0};
  std::vector<std::vector<float>> lat(nthreads);
  const auto t_end = Clock::now() + std::chrono::microseconds((long long)(secs * 1e6));
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
      if (connect(fd, (sockaddr*)&a, sizeof a) != 0) { errors++; close(fd); cs[i].fd = -1; continue; }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      cs[i].fd = fd;
      epoll_event e{};
      e.events = EPOLLIN;
      e.data.u32 = (uint32_t)i;
      epoll_ctl(ep, EPOLL_CTL_ADD, fd, &e);
      cs[i].t0 = Clock::now();
      if (write(fd, req.data(), req.size()) != (ssize_t)req.size()) errors++;
    }
    std::vector<float>& L = lat[tid];
    epoll_event evs[512];
    char buf[1 << 16];
    while (Clock::now() < t_end) {
      const int n = epoll_wait(ep, evs, 512, 50);
      for (int k = 0; k < n; ++k) {
        C& c = cs[evs[k].data.u32];
        const ssize_t r = read(c.fd, buf, sizeof buf);
        if (r <= 0) { errors++; continue; }
        c.in.append(buf, (size_t)r);
        while (true) {
          const size_t h = c.in.find("\r\n\r\n");
          if (h == std::string::npos) break;
          size_t clen = 0;
          const size_t cl = c.in.find("content-length:");
          if (cl != std::string::npos && cl < h) clen = std::strtoull(c.in.c_str() + cl + 15, nullptr, 10);
          if (c.in.size() < h + 4 + clen) break;
          if (c.in.compare(0, 12, "HTTP/1.1 200") != 0) errors++;
          c.in.erase(0, h + 4 + clen);
          const auto now = Clock::now();
          L.push_back((float)std::chrono::duration<double, std::micro>(now - c.t0).count());
          total++;
          if (now < t_end) {
            c.t0 = now;
            if (write(c.fd, req.data(), req.size()) != (ssize_t)req.size()) errors++;
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
  const double el = std::chrono::duration<double>(Clock::now() - t0).count();
  std::vector<float> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : (double)all[std::min(all.size() - 1, (size_t)(p * all.size()))]; };
  std::printf("{\"connections\": %d, \"threads\": %d, \"seconds\": %.2f, \"requests\": %lld, \"req_per_s\": %.1f, "
              "\"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, \"errors\": %lld, \"body_bytes\": %zu}\n",
              nconn, nthreads, el, total.load(), total.load() / el, pct(0.5), pct(0.9), pct(0.99),
              all.empty() ? 0.0 : (double)all.back(), errors.load(), body.size());
  return 0;
}
