// Host-side launcher declarations for every routest_amd HIP kernel (gfx950).
#pragma once
#include <memory>
#include <hip/hip_runtime.h>

#include <string>
#include <vector>
#include <stddef.h>
#include <stdint.h>

namespace rt {

struct NormParams;

// ---- ETA MLP (K1 featurize + K2 forward) : eta_mlp_fwd.hip ----
size_t eta_mlp3_blob_bytes(int H);
// variant: -1 auto, 0 weights from global/L2, 1 weights staged in LDS (persistent grid)
hipError_t launch_eta_mlp3_fwd(const void* rec, float* out, int B, const void* blob, int H,
                               const NormParams& np, int variant, int num_cus, hipStream_t stream,
                               int rec_bytes = 16);   // 16, 8 or 6-byte records
// 16x16-MFMA form (blob16 layout, ops/eta_mlp.py pack_mlp3_16); nh = 1, 2 or 4 batch halves
size_t eta_mlp3_blob16_bytes(int H);
hipError_t launch_eta_mlp3_fwd16(const void* rec, float* out, int B, const void* blob16, int H,
                                 const NormParams& np, int nh, int num_cus, hipStream_t stream,
                                 int rec_bytes);
hipError_t launch_eta_featurize(const void* rec, float* out, int B, hipStream_t stream);

// ---- ETA MLP training (K3) : eta_mlp_train.hip ----
// forward + MSE gradient in one pass over layer 2; writes xf [ceil(B/32)*32, 16] (rows past B
// untouched), the dz2 fragments ([ceil(B/32)][H/16][64] x 16 bytes, train_bwd_kernel's A-operand
// order), squared errors and the dW3 slab
hipError_t launch_eta_mlp3_train_fwd(const void* rec, const float* target, int B, const void* blob,
                                     int H, const NormParams& np, float gscale, void* xf,
                                     float* w3slab, void* dz2r, float* sq_err, int* step_ctr, int num_cus,
                                     hipStream_t stream);
int train_fwd_grid(int B, int num_cus);   // workgroups = rows of the dW3 slab
// dgrad + relu'(z1) + dW2|db2 and dW1 partials per k-slice (slab2 [S][H][H+16], slab1 [S][H][16],
// bucket order); xf must hold ceil(B/32)*32 rows (zeros past B)
hipError_t launch_train_bwd(const void* xf, int B, const void* blob, int H, const void* dz2r, float* slab2,
                            float* slab1, int S, hipStream_t stream);
int train_wgrad_slices(int B, int num_cus, int H = 256);
size_t eta_mlp3_train_blob_bytes(int H);
int mlp3_num_params(int H);
int mlp3_grad_bucket_floats(int H);
hipError_t launch_adamw_pack(float* P, const float* G, float* M, float* V, void* blob,
                             const int* step, int H, float lr, float beta1, float beta2, float eps,
                             float wd, int warmup, int total_steps, float min_lr_ratio, int update,
                             hipStream_t stream);
// one-rank fused wgrad_reduce (dW2 register-native slabs | dW1 slabs | dW3 rows) + adamw_pack(update)
hipError_t launch_reduce_adamw(const float* slab2, int S2, long long stride2, const float* slab1, int S1,
                               long long stride1, const float* w3slab, int S3, long long stride3, float* G,
                               float* P, float* M, float* V, void* blob, const int* step, int H, float lr,
                               float beta1, float beta2, float eps, float wd, int warmup, int total_steps,
                               float min_lr_ratio, hipStream_t stream);

// ---- wide MLPs (H = 512, 1024): mlp_big.hip ----
hipError_t launch_big_layer1(const void* rec, int rec_bytes, int B, const void* w1p, int H,
                             const NormParams& np, void* h1, int ld, void* xf, hipStream_t stream,
                             unsigned* mbits = nullptr);
// training dgrad dh1 = dz2 W2 with dW1 = (dh1 * relu'(z1))^T xf in its epilogue (dh1 never stored;
// mbits: big_layer1's relu bit mask [M][N/32]):
// slab1 [ceil(M / 256)][>= 16 N] f32 partials per 256-row tile (mlp_big.hip EPI_DW1)
hipError_t launch_gemm_dgrad_dw1(const void* W, int ldw, const void* X, int ldx, int N, int M, int K,
                                 const unsigned* mbits, const void* xf, float* slab1, long long slab1_ld,
                                 hipStream_t stream);
hipError_t launch_gemm_nt(int epi, const void* W, int ldw, const void* X, int ldx, int N, int M,
                          int K, const float* b2, const float* w3, float* ypart, void* out,
                          int ldo, hipStream_t stream);
// K loop of the 256 x 256 wide GEMM: 1 phase pipeline (default), 0 one drain per K-tile; < 0 only reads
int gemm_pipe_mode(int set = -1);
hipError_t launch_big_fused(const void* rec, int rec_bytes, int B, const void* w1q, const void* w2f,
                            int H, const NormParams& np, const float* b2, const float* w3,
                            float* ypart, hipStream_t stream);
hipError_t launch_big_yreduce(const float* ypart, int nparts, int B, float b3, const float* b3p,
                              float* y, const float* target, float gscale, float* dy, void* dyb,
                              float* sq_err, hipStream_t stream);
hipError_t launch_adamw_pack_big(float* P, const float* G, float* M, float* V, void* w1p, void* w2k,
                                 void* w2t, float* b2, float* w3, float* b3, const int* step, int H,
                                 float lr, float beta1, float beta2, float eps, float wd, int warmup,
                                 int total_steps, float min_lr_ratio, int update, hipStream_t stream);
hipError_t launch_big_dz2y(const float* ypart, int nparts, int B, int H, const float* b3p,
                           const float* target, float gscale, float* dy, void* dyb, float* sq_err,
                           const void* h2a, int lda, const float* w3, void* dz2, int* step_ctr,
                           hipStream_t stream);
// + dW3 | db3: slab[s][0 .. H+16) for s < S (H = 512 or 1024)
hipError_t launch_big_dz2y_w3(const float* ypart, int nparts, int B, int H, const float* b3p,
                              const float* target, float gscale, float* dy, void* dyb, float* sq_err,
                              const void* h2a, int lda, const float* w3, void* dz2, int* step_ctr, float* slab,
                              long long slab_ld, int S, hipStream_t stream);
hipError_t launch_big_dz2(const void* h2a, int lda, const float* dy, const float* w3, int B, int H,
                          void* dz2, hipStream_t stream);

// ---- weight-gradient GEMMs with K = batch : wgrad.hip ----
hipError_t launch_wgrad(const void* A, int lda, int M, int Mout, const void* Bm, int ldb, int N,
                        int K, int S, float* slab, int ldo, long long slab_stride, hipStream_t stream,
                        const void* mask = nullptr, int ldm = 0, int Nout = -1,
                        bool mask_hperm = false, int nsplit = 1);
hipError_t launch_wgrad_reduce(const float* slab, int S, long long slab_stride, float* G, int n,
                               hipStream_t stream, const float* slab1 = nullptr, int S1 = 0,
                               long long slab_stride1 = 0, float* G1 = nullptr, int n1 = 0,
                               const float* slab2 = nullptr, int S2 = 0, long long slab_stride2 = 0,
                               float* G2 = nullptr, int n2 = 0, int perm_h0 = 0, int fold_ld0 = 0,
                               int fold_col0 = 0);
// dW2-shaped weight gradient on 256 x 256 output tiles, split-K over S slices (wgrad.hip); db2_col >= 0:
// column sums of A into slab columns db2_col .. db2_col + N/256 - 1 (fold them with wgrad_reduce)
hipError_t launch_wgrad256(const void* A, int lda, const void* B, int ldb, int M, int N, int K, int S, float* slab,
                           int ldo, long long slab_stride, int db2_col, hipStream_t stream);
size_t wgrad_lds_bytes(int NT);
// two independent wgrad GEMMs (segment 1: N <= 32) in one launch, same K
hipError_t launch_wgrad_dual(const void* A0, int lda0, int M0, int Mout0, const void* B0, int ldb0,
                             int N0, int K, int S0, float* slab0, int ldo0, long long stride0, int Nout0,
                             int nsplit0, const void* A1, int lda1, int M1, int Mout1, const void* B1,
                             int ldb1, int N1, int S1, float* slab1, int ldo1, long long stride1,
                             int Nout1, hipStream_t stream);

// ---- GCN route scorer (K8) : gcn.hip ----
hipError_t launch_gcn_agg_gemm(const void* X, const int* indptr, const int* indices,
                               const float* values, const void* wfrag, const float* bias, void* Y,
                               int fin, int fout, bool agg, bool relu, int row0, int row1,
                               int num_cus, hipStream_t stream);
hipError_t launch_gcn_l1_fused(const void* X, const int* indptr, const int* indices, const float* values,
                               const void* w1frag, const float* b1, const void* w2frag, void* Z, int fin,
                               int fhid, int fz, int row0, int row1, int num_cus, hipStream_t stream);
hipError_t launch_gcn_spmm_score(const void* Z, const int* indptr, const int* indices,
                                 const float* values, const float* b2, const float* wo, float bo,
                                 float* delay, int row0, int row1, hipStream_t stream);
hipError_t launch_route_score(const int* rptr, const int* nodes, const float* latlon,
                              const float* delay, float* score, int R, int N, hipStream_t stream);

// ---- GCN scorer training (K8 backward) : gcn_train.hip ----
int gcn_grad_numel();
int gcn_train_slab2_rows(int N);
hipError_t launch_gcn_train_bwd(const void* X, const void* Z, const int* indptr, const int* indices,
                                const float* values, const void* w1frag, const float* b1, const float* W2,
                                const float* b2, const float* wo, const float* bo, const float* target, int N,
                                int r0, int r1, float* dy, float* slab1, int slab1_rows, float* slab2,
                                float* grad, float* loss, int num_cus, hipStream_t stream);

// ---- batched A* (K9) : astar.hip ----
// Device graph (CSR + coordinates + ALT tables) as the kernels read it.
struct AstarGraphDev {
  const int* indptr = nullptr;
  const int* indices = nullptr;
  const float* cost = nullptr;
  const float* lat = nullptr;
  const float* lon = nullptr;
  int N = 0;
  float inv_vmax = 0.f;
  const float* lm = nullptr;   // [N][2K] or nullptr
  int K = 0;
};
// One tier's workspace: `slots` searches, each with a hash table of 1 << tbits 16-byte entries
// (all-ones when idle), a heap row of `cap` u64 and a reset list of (1 << tbits) / 2 ints.
struct AstarWs {
  void* tab = nullptr;
  void* heap = nullptr;
  int* touched = nullptr;
  int slots = 0, cap = 0, tbits = 0;
};
// Growth arena of the wave/big tiers: `entries` 16-byte entries, all-ones when idle, and an 8-byte
// device bump counter (the launcher resets it before every wave launch).
struct AstarArenaBuf {
  void* base = nullptr;
  unsigned long long entries = 0;
  unsigned long long* ctr = nullptr;
};
struct AstarOut {
  float* cost = nullptr;
  int* len = nullptr;
  int* status = nullptr;    // 0 found, 1 unreachable, 2 overflow, 3 max_iters, 4 path > max_path
  int* path = nullptr;      // [Q][max_path]
  int max_path = 0;
  int* iters = nullptr;     // [Q] or nullptr
};
struct AstarPlan {
  int max_iters = 2000000;
  int lane_pops = 500;          // <= 0: lane tier only, run to max_iters
  int wave_only_below = 32768;  // fewer queries than this: skip the lane tier
  float delta = 10.f;           // wave tier f-band width (seconds)
  float lane_max_m = -1.f;      // legs longer than this (great circle, m) skip the lane tier; 0: none;
                                // < 0: ROUTEST_ASTAR_LANE_MAX_M, read per search (default 0)
  int wave_nw = 0;              // waves per search in the main wave-tier launch (1, 2, 4, 8);
                                // 0: ROUTEST_ASTAR_WAVE_WAVES, read per search (default 1)
  int retry_nw = 0;             // waves per search in the arena reruns and the big tier;
                                // 0: ROUTEST_ASTAR_RETRY_WAVES, read per search (default 4)
};
struct AstarRunStats {
  int lane = 0, wave = 0, escalated = 0;
  double lane_ms = 0, wave_ms = 0, big_ms = 0;
  int retried = 0;              // wave-tier overflows rerun a few at a time (larger arena share)
  double retry_ms = 0;
};
bool astar_ws_ok(const AstarWs& ws, bool wave);
hipError_t launch_astar_lane(const AstarGraphDev& g, const int* src, const int* dst, int Q, int q0,
                             const AstarWs& ws, const AstarOut& o, int max_iters, hipStream_t stream,
                             const int* qidx = nullptr, int nq = 0);   // qidx: run queries qidx[0..nq)
hipError_t launch_astar_wave(const AstarGraphDev& g, const int* src, const int* dst, int Q, const int* qidx,
                             int q0, int T, const AstarWs& ws, const AstarOut& o, int max_iters, float delta,
                             hipStream_t stream, const AstarArenaBuf* arena = nullptr,
                             int nw = 1);   // nw: waves per search (1, 2, 4 or 8)
// The tiered search (lane -> wave -> big); any tier pointer may be null.  scratch: Q + 1 device ints.
// Searches left with status 2/3 are the caller's (host Dijkstra).
hipError_t astar_search(const AstarGraphDev& g, const int* src, const int* dst, int Q, const AstarWs* lane,
                        const AstarWs* wave, const AstarWs* big, const AstarOut& o, const AstarPlan& pl,
                        int* scratch, hipStream_t stream, AstarRunStats* st,
                        const AstarArenaBuf* arena = nullptr);

// ---- tree ensemble (K4) : forest.hip ----
hipError_t launch_forest(const void* rec, const float* values, const unsigned* info, const int* roots,
                         float* out, int B, int T, int M, float base, int le, const int* fmap,
                         hipStream_t stream);

hipError_t launch_forest_lds(const void* rec, const void* nodes2, const int* roots, const int* chunks,
                             int nchunks, float* out, int B, int T, int M, float base, int le,
                             const int* fmap, int num_cus, hipStream_t stream);

// ---- batched routing (K5 distance matrix + K6 greedy CVRP) : route_kernels.hip ----
hipError_t launch_haversine_matrix(const double* lat, const double* lon, const int* npts, int R,
                                   int NM, double circuity, double* D, hipStream_t stream);
hipError_t launch_greedy_cvrp(const double* D, const int* npts, const double* demand,
                              const double* cap, const double* maxd, int R, int NM, int* visit,
                              int* trip_of, int* ntrips, int* status, hipStream_t stream);

// ---- persistent single-request scorer : persistent_serve.hip ----
struct PersistentScorer;
PersistentScorer* pscore_create(int device, const void* blob, int H, const NormParams& np, int cap,
                                double idle_ms, double life_ms, hipError_t* err);
void pscore_park(PersistentScorer* s);
void* pscore_records(PersistentScorer* s);
const float* pscore_out(PersistentScorer* s);
int pscore_cap(PersistentScorer* s);
bool pscore_broken(PersistentScorer* s);
void pscore_stats(PersistentScorer* s, long long* launches, long long* served, long long* fallbacks);
hipError_t pscore_run(PersistentScorer* s, int n, double timeout_ms);
void pscore_destroy(PersistentScorer* s);

// ---- native front end (predictions, routes, relay to the Python app) : native_server.hip ----
struct RouteServiceCfg;   // route_service.h
struct NativeModel;       // native_model.h
int64_t native_server_start(int port, int threads, const std::vector<int>& devices,
                            const std::vector<std::shared_ptr<const NativeModel>>& models, int max_batch,
                            const std::vector<std::string>& cors, bool cors_vercel, bool bind_any, int upstream_port,
                            const std::vector<RouteServiceCfg>& routes, const std::string& history_db,
                            std::string& err);
int64_t native_server_set_models(int64_t h, const std::vector<std::shared_ptr<const NativeModel>>& models,
                                 std::string& err);
bool native_server_set_fault(int64_t h, int slot, bool on);
bool native_server_set_hang(int64_t h, int slot, bool on);
bool native_server_set_scorer(int64_t h, std::vector<double> delay, int kind, const std::string& engine);
std::vector<std::vector<std::string>> native_server_health(int64_t h, uint64_t& epoch);
void native_server_stop(int64_t h);
std::vector<long long> native_server_stats(int64_t h);

// ---- native collectives (rccl_ops) : comm.hip ----
int comm_unique_id(char out[128]);
int64_t comm_create(const char* uid, int rank, int world, int device, size_t oneshot_bytes, bool use_rccl,
                    std::string& errmsg);
int comm_ipc_handle_bytes();
int comm_ipc_handles(int64_t h, char* out);
int comm_open_peers(int64_t h, const std::vector<std::string>& handles, std::string& errmsg);
hipError_t comm_all_reduce_f32(int64_t h, float* data, size_t n, int algo, hipStream_t stream,
                               std::string& errmsg);
int comm_nccl_call(int64_t h, int op, const void* in, void* out, size_t count, int dtype, int root,
                   hipStream_t stream, std::string& errmsg);
hipError_t comm_all_gather_oneshot(int64_t h, const void* in, void* out, size_t bytes_per_rank,
                                   hipStream_t stream, std::string& errmsg);
hipError_t comm_broadcast_oneshot(int64_t h, void* data, size_t bytes, int root, hipStream_t stream,
                                  std::string& errmsg);
int comm_error(int64_t h);
int comm_world(int64_t h);
void comm_destroy(int64_t h);
int comm_rccl_version();

}  // namespace rt
