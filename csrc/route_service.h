// Native route service (csrc/route_service.hip): request/response types shared with the native
// front end (csrc/native_server.hip).
#pragma once
#include <cmath>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "cch_gpu.h"
#include "common.h"
#include "native_model.h"
#include "ops.h"
#include "runtime/route_core.h"
#include "runtime/route_record.h"

#include <mutex>

namespace rt {

struct PersistentScorer;
struct RouteJob;

// A stream on a hardware queue of its own (a full CU mask makes the runtime give the stream a
// dedicated queue): the gpu_hang fault hook runs the hung work on one, so on a shared-GPU
// rehearsal the other slot's streams are never queued behind it — on a real node the slots are
// separate GPUs anyway.
inline hipError_t isolated_stream(int device, hipStream_t* s) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xFFFFFFFFu);
  return hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
}

// The GCN candidate-route scorer's node delay factors for "alternatives" requests
// (routing/alternatives.py; csrc/runtime/alternatives.h), published by the Python side once the
// scorer is trained (NativePredictServer.set_scorer); until then such requests go to the app.
struct AltScorerState {
  std::mutex mu;
  std::shared_ptr<const std::vector<double>> delay;   // [N] delay factor per graph node
  int kind = 0;                                       // ralt::OBSERVED / EDGE
  std::string engine = "gcn-hip";                     // RouteScorer.engine
  std::shared_ptr<const std::vector<double>> get(int& k, std::string& e) {
    std::lock_guard<std::mutex> lk(mu);
    k = kind;
    e = engine;
    return delay;
  }
};

struct RouteServiceCfg {
  int device = 0;
  int provider = 0;                       // 0 haversine, 1 road graph (A* or CCH)
  // road graph through the customizable contraction hierarchy (csrc/cch.hip): when set, the road
  // matrices, the greedy's trips and every leg come from it, under each request's routing context
  // (or one fixed metric when cch_contexts is false); the A* fields below are then unused
  CchGpu* cch = nullptr;
  bool cch_contexts = true;
  uint64_t cch_fixed_key = 0;
  const float* h_length = nullptr;        // [E] metres per edge (maneuvers)
  const int32_t* h_edge_name = nullptr;   // [E] road name ids (-1 unnamed), optional
  std::vector<std::string> names;         // road name table
  double circuity = 1.3, step_m = 150.0;  // HaversineProvider (routing/providers.py)
  std::string engine = "backend:mi355x";
  bool compat200 = true;                  // /api/request_route answers errors with 200 (reference)
  int batch_max = 1024;
  double timeout_us = 500.0;
  int chunk_threads = 16;                 // host fan-out per parallel_chunks call (assembly, legs)
  // road graph, host side (assembly, snapping, exact fallback)
  const double* glat = nullptr;
  const double* glon = nullptr;
  int N = 0;
  double snap_c = 1.0;
  const int* h_indptr = nullptr;
  const int* h_indices = nullptr;
  const float* h_cost = nullptr;
  // road graph, device side (routing/graph.py BatchedAstar's tensors)
  const int* indptr = nullptr;
  const int* indices = nullptr;
  const float* cost = nullptr;
  const float* lat32 = nullptr;
  const float* lon32 = nullptr;
  const float* lm = nullptr;
  int K = 0;
  AstarWs lane_ws, wave_ws, big_ws;       // the tiers' workspaces (csrc/astar.hip); slots == 0: off
  AstarArenaBuf arena;                    // growth arena of the wave/big tiers (optional)
  int max_path = 4096, max_iters = 2000000, lane_pops = 500;
  int wave_only_below = 32768;            // fewer unique legs than this: every search in the wave tier
  float inv_vmax = 0.f, wave_delta = 10.f, lane_max_m = -1.f;
  // ETA model for use_ml_eta: the native front end's current model of this GPU slot (hot-swapped)
  std::function<std::shared_ptr<const NativeModel>()> eta_model;
  // persistence: SQLite database path/URI of the Python store ("" = none)
  std::string sqlite_path;
  // parks the GPU's resident single-request scorer (persistent_serve.hip) before each flush's
  // launches so they never queue behind it on a shared hardware queue
  std::function<void()> park_scorer;
  // GCN scorer for "alternatives" requests (road graph + CCH only)
  std::shared_ptr<AltScorerState> alt;
  // latency watchdog (ROUTEST_ROUTE_DEADLINE_MS): a flush whose GPU work misses the deadline marks
  // the service broken until that work drains; its jobs — and every flush meanwhile — are handed
  // to `failover` (another GPU's route service; false: none left -> relayed to the app).  A job is
  // handed on at most n-1 times (RouteJob::hops): a failure that repeats on every service (an
  // allocation, a context build) ends at the app instead of bouncing between services forever
  //
  std::function<bool(RouteJob*)> failover;
  // the road graph's compact-record view (csrc/runtime/route_record.h), shared with the native
  // history readers; unset: the service builds its own when the graph carries edge metres
  std::shared_ptr<const rrec::RecordGraph> record_graph;
  std::function<void()> on_timeout;       // the slot's GPU is quarantined for predictions too
  int slot = -1;                          // the server's slot (traces: ROUTEST_ROUTE_TRACE_MS)
  std::function<bool()> hang_fault;       // ROUTEST_FAULT=gpu_hang@<slot> (the watchdog's test hook)
  const int* hang_release_d = nullptr;    // its device-visible release flag
};

// One request handed from a reactor to the service and back.
struct RouteJob {
  std::string body;                 // request body
  bool json_ok = true;              // content-type is JSON
  bool request_route = false;       // /api/request_route (non-silent JSON, never persisted)
  void* tag = nullptr;              // reactor-owned context
  // result: fallback (hand to the Python app) or status + bytes
  bool fallback = false;
  int status = 0;
  std::string out;
  // internal
  rtj::Value root;
  rtr::RouteReq req;
  rtr::Plan plan;
  std::vector<std::vector<std::pair<double, double>>> calls;
  std::vector<int32_t> nodes;
  int group = 0;                    // routing-context group of its flush (CCH)
  bool parsed = false;              // request parsed (a job deferred for its context keeps it)
  double defer_t0 = 0.0;            // when it was first deferred for its context's build (us)
  bool sync_ctx = false;            // its context's background build failed: build it in the flush
  int hops = 0;                     // times handed to another GPU's route service (failover)
  double t_enq_us = 0.0;            // when it entered the flush queue (steady clock, us)
  // "alternatives": unique leg pairs in order, their via nodes, the chosen candidates (legs owned
  // here) and the response block
  std::vector<std::pair<int, int>> alt_pairs;
  std::vector<std::vector<int>> alt_vias;
  std::vector<rtr::Leg> alt_legs;
  std::vector<std::vector<int32_t>> alt_paths, alt_edges;
  std::string alt_json;
  rtr::Assembled asmb;
  float eta_min = NAN;
  std::string eta_iso, request_id;
  std::string p_stops, p_geom;      // row texts for the persistence thread (prep_persist)
  std::string rec;                  // compact route record (route_record.h; "" = legs / geometry as text)
  bool p_ok = false;
  rtc::Stamp now;
};

class RouteService {
 public:
  RouteService(const RouteServiceCfg& cfg, std::function<void(RouteJob*)> done);
  ~RouteService();
  // false once the service is stopping (the job is not taken: the caller relays it to the app)
  bool submit(RouteJob* j);
  // finished jobs handed back many at a time (one wake-up per receiver instead of one per job);
  // set before the first submit.  Unset: `done` per job.
  void set_done_batch(std::function<void(std::vector<RouteJob*>&)> done_many);
  // jobs, flushes, fallbacks, legs searched, legs finished on the host, rows persisted
  std::vector<long long> stats() const;
  bool broken() const;                    // a flush missed the deadline and its GPU work has not drained

 private:
  struct Impl;
  Impl* p_;
};

}  // namespace rt
