// Closed-loop HTTP/1.1 load generator for the prediction endpoints (wrk is not in the image).
//
//   loadgen <port> <connections> <seconds> [path] [body-file|-] [threads]
//
// Each connection keeps one request in flight (keep-alive); responses are parsed by
// Content-Length (runtime/http_client.h).  Prints one JSON line: requests/s, latency
// p50/p90/p99/max (us), errors.
#include <cstdio>
#include <fstream>
#include <sstream>

#include "../runtime/http_client.h"

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
  const rtc::LoadResult r = rtc::http_load(port, nconn, secs, path, body, nthreads);
  std::printf("{\"connections\": %d, \"threads\": %d, \"seconds\": %.2f, \"requests\": %lld, \"req_per_s\": %.1f, "
              "\"p50_us\": %.1f, \"p90_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, \"errors\": %lld, \"body_bytes\": %zu}\n",
              nconn, nthreads, r.seconds, r.requests, r.requests / r.seconds, r.pct(0.5), r.pct(0.9), r.pct(0.99),
              r.lat_us.empty() ? 0.0 : (double)r.lat_us.back(), r.errors, body.size());
  return 0;
}
