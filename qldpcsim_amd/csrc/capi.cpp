// capi.cpp — C ABI (include/qldpc_decoder.h): Tanner-graph preparation,
// schedules, kernel launch configuration, host staging and timing.
//
// Replaces the per-call setup the reference repeats for every shot:
//   BP_decoder's edge lists   np.where(H) + per-check/per-var lists  decoders.py:224-229
//   MS_decoder's dense masks  H == 1 over m x n                       decoders.py:148-169
// Here the graph is built once per H, bit-exactly ordered (CSR edges in
// np.where(H) order; CSC lists in ascending check order), relabeled so that
// variables of equal degree share wavefront passes, and uploaded once.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <thread>
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qldpc_decoder.h"
#include "../../include/qldpc_libm.h"
#include "decoder_kernels.h"
#include "osd_kernels.h"
#include "channel_kernels.h"
#include "hbm_kernels.h"
#include "tuning.h"

using qldpc::DecodeArgs;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(QLDPC_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),    \
                  __FILE__, __LINE__);                                                  \
  } while (0)

extern "C" const char* qldpc_last_error(void) { return g_err.c_str(); }
extern "C" const char* qldpc_version(void) { return "qldpcsim_amd 0.1.0 (gfx950)"; }

extern "C" int qldpc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ---------------------------------------------------------------------------
// options (include/qldpc_decoder.h): read at launch, never from the
// environment; `gen` changes with every set so cached launch configurations
// are rebuilt
// ---------------------------------------------------------------------------
namespace {
struct Options {
  std::atomic<int64_t> force_hbm{0}, flood_generic{0}, layered_generic{0}, ms_lanes_per_check{0}, bp_wave{0},
      bp_lg{1}, bp_team_w{0}, static_sched{0}, waves_per_wg{0}, wg_per_cu{0}, osd_column{0}, osd_tickets{1},
      osd_prof{0}, osd_hbm{0};
  std::atomic<uint32_t> gen{1};
};
Options g_opt;

std::atomic<int64_t>* option_slot(const char* name) {
  if (!name) return nullptr;
  static const struct {
    const char* name;
    std::atomic<int64_t> Options::*slot;
  } table[] = {{"force_hbm", &Options::force_hbm},     {"flood_generic", &Options::flood_generic},
               {"layered_generic", &Options::layered_generic},
               {"ms_lanes_per_check", &Options::ms_lanes_per_check},
               {"bp_wave", &Options::bp_wave},         {"bp_lg", &Options::bp_lg},
               {"bp_team_w", &Options::bp_team_w},     {"static_sched", &Options::static_sched},
               {"waves_per_wg", &Options::waves_per_wg}, {"wg_per_cu", &Options::wg_per_cu},
               {"osd_column", &Options::osd_column},   {"osd_tickets", &Options::osd_tickets},
               {"osd_prof", &Options::osd_prof},       {"osd_hbm", &Options::osd_hbm}};
  for (const auto& e : table)
    if (strcmp(e.name, name) == 0) return &(g_opt.*(e.slot));
  return nullptr;
}

int64_t opt(std::atomic<int64_t> Options::*slot) { return (g_opt.*slot).load(std::memory_order_relaxed); }
}  // namespace

extern "C" int qldpc_set_option(const char* name, int64_t value) {
  std::atomic<int64_t>* o = option_slot(name);
  if (!o) return fail(QLDPC_EINVAL, "unknown option %s", name ? name : "(null)");
  o->store(value);
  g_opt.gen.fetch_add(1);
  return QLDPC_OK;
}

extern "C" int qldpc_get_option(const char* name, int64_t* value) {
  std::atomic<int64_t>* o = option_slot(name);
  if (!o || !value) return fail(QLDPC_EINVAL, "unknown option %s", name ? name : "(null)");
  *value = o->load();
  return QLDPC_OK;
}

// ---------------------------------------------------------------------------
// code (Tanner graph)
// ---------------------------------------------------------------------------
struct qldpc_code {
  int m = 0, n = 0, E = 0, device = 0;
  int uniform_deg = 0;  // row degree if every row has it, else 0
  int max_row_deg = 0, max_col_deg = 0;
  // GF(2) rank of H (gf2math.rank) and column bit-vectors, for OSD only:
  // built on first use (code_osd_prep), a large code may never need them
  mutable std::once_flag osd_once;
  mutable int rank = -1;
  bool zero_col = false;  // H has an all-zero column (GPU OSD: exact REF kernel only)
  // the LDS-resident kernels' 16-bit tables hold this code (m, n, E <= 65535);
  // otherwise every decode takes the HBM-resident kernel
  bool lds_ok = true;
  std::vector<int32_t> row_ptr, col_idx;     // CSR, np.where(H) order
  std::vector<int32_t> vperm, vinv;          // relabeled -> original, original -> relabeled
  std::vector<int32_t> csc_ptr, csc_edge;    // relabeled-variable CSC: CSR edge ids, ascending check
  std::vector<int32_t> edge_pos;             // CSR edge -> CSC position
  int mw = 0;                                // 64-bit words per column bit-vector
  mutable std::vector<uint64_t> col_bits;    // [n][mw] column j of H (OSD)
  uint16_t* d_vinv = nullptr;
  // HBM-resident kernel: 32-bit graph tables (relabeled variables)
  int32_t *d_row_var = nullptr, *d_row_pos = nullptr, *d_col_ptr = nullptr, *d_vinv32 = nullptr;
  int32_t *d_row_ptr = nullptr, *d_col_idx = nullptr;  // CSR for the GPU OSD
  // layered MS stop-test filters (ms_layered_kernel): 32 fixed random parity
  // checks of H's rows; wc[c] bit k = row c in check k, avar[v] bit k = parity
  // of the rows of check k that hold relabeled variable v
  std::vector<uint32_t> wc, avar;
  uint32_t filt_all = 0;
  uint32_t *d_wc = nullptr, *d_rtab = nullptr;  // rtab: [m][8] relabeled variables per row
  uint32_t* d_avar = nullptr;                    // [n] filter word per relabeled variable (layered BP)
  // host staging workspace for qldpc_decode_host: device buffers, page-locked
  // host mirrors (DMA copies) and a stream of its own (no device-wide sync)
  std::mutex ws_mu;
  int64_t ws_cap = 0;
  uint8_t *ws_syn = nullptr, *ws_ehat = nullptr;
  int32_t *ws_iters = nullptr, *ws_flags = nullptr;
  double* ws_post = nullptr;
  uint8_t *hp_syn = nullptr, *hp_ehat = nullptr;
  int32_t *hp_iters = nullptr, *hp_flags = nullptr;
  double* hp_post = nullptr;
  hipStream_t ws_stream = nullptr;
};

static int gf2_rank_cols(const std::vector<uint64_t>& cols, int n, int mw);

extern "C" int qldpc_code_create(const uint8_t* h_H, int m, int n, qldpc_code** out) {
  if (!out) return fail(QLDPC_EINVAL, "out is null");
  *out = nullptr;
  if (m < 0 || n < 0 || (m * (int64_t)n > 0 && !h_H)) return fail(QLDPC_EINVAL, "bad shape %d x %d", m, n);
  auto* c = new qldpc_code();
  c->m = m;
  c->n = n;
  // No visible device (e.g. the CPU build container): the graph is still built
  // so host-side services (OSD) work; decode entry points then fail loudly.
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || hipGetDevice(&c->device) != hipSuccess)
    c->device = -1;
  c->row_ptr.assign(m + 1, 0);
  for (int r = 0; r < m; ++r) {
    for (int j = 0; j < n; ++j)
      if (h_H[(size_t)r * n + j] & 1) c->col_idx.push_back(j);  // (mat % 2) (simulator.py:35)
    c->row_ptr[r + 1] = (int32_t)c->col_idx.size();
  }
  c->E = (int)c->col_idx.size();
  c->lds_ok = m <= 65535 && n <= 65535 && c->E <= 65535;
  std::vector<int> cdeg(n, 0);
  for (int e = 0; e < c->E; ++e) cdeg[c->col_idx[e]]++;
  for (int r = 0; r < m; ++r) c->max_row_deg = std::max(c->max_row_deg, c->row_ptr[r + 1] - c->row_ptr[r]);
  for (int j = 0; j < n; ++j) c->max_col_deg = std::max(c->max_col_deg, cdeg[j]);
  c->uniform_deg = m > 0 ? c->row_ptr[1] : 0;
  for (int r = 0; r < m; ++r)
    if (c->row_ptr[r + 1] - c->row_ptr[r] != c->uniform_deg) c->uniform_deg = 0;
  // Relabel variables by degree (stable) so a wavefront pass over 64
  // consecutive relabeled variables has (nearly) one loop trip count.
  c->vperm.resize(n);
  for (int j = 0; j < n; ++j) c->vperm[j] = j;
  std::stable_sort(c->vperm.begin(), c->vperm.end(), [&](int a, int b) { return cdeg[a] < cdeg[b]; });
  c->vinv.resize(n);
  for (int r = 0; r < n; ++r) c->vinv[c->vperm[r]] = r;
  // CSC over relabeled variables; CSR traversal in ascending row keeps each
  // column's list in ascending check order (np.sum axis=0 order).
  c->csc_ptr.assign(n + 1, 0);
  for (int r = 0; r < n; ++r) c->csc_ptr[r + 1] = c->csc_ptr[r] + cdeg[c->vperm[r]];
  c->csc_edge.assign(c->E, 0);
  c->edge_pos.assign(c->E, 0);
  std::vector<int32_t> fill(c->csc_ptr.begin(), c->csc_ptr.end() - 1);
  for (int r = 0; r < m; ++r)
    for (int e = c->row_ptr[r]; e < c->row_ptr[r + 1]; ++e) {
      const int pos = fill[c->vinv[c->col_idx[e]]]++;
      c->csc_edge[pos] = e;
      c->edge_pos[e] = pos;
    }
  c->mw = (m + 63) / 64;
  for (int j = 0; j < n && !c->zero_col; ++j) c->zero_col = cdeg[j] == 0;
  c->wc.resize(m);
  for (int r = 0; r < m; ++r) {
    uint64_t z = 0x9E3779B97F4A7C15ull * (uint64_t)(r + 1) + 0xD1B54A32D192ED03ull;   // splitmix64
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    c->wc[r] = (uint32_t)((z ^ (z >> 31)) >> 16);
  }
  c->avar.assign(n, 0);
  for (int r = 0; r < m; ++r)
    for (int e = c->row_ptr[r]; e < c->row_ptr[r + 1]; ++e) c->avar[c->vinv[c->col_idx[e]]] ^= c->wc[r];
  for (int v = 0; v < n; ++v) c->filt_all ^= c->avar[v];
  if (n > 0 && c->device >= 0) {
    hipError_t e1 = hipSuccess;
    if (c->lds_ok) {
      std::vector<uint16_t> v16(c->vinv.begin(), c->vinv.end());
      e1 = hipMalloc(&c->d_vinv, sizeof(uint16_t) * n);
      if (e1 == hipSuccess) e1 = hipMemcpy(c->d_vinv, v16.data(), sizeof(uint16_t) * n, hipMemcpyHostToDevice);
    }
    {  // HBM-resident kernel tables
      std::vector<int32_t> rv(std::max(c->E, 1)), rp(std::max(c->E, 1));
      for (int e = 0; e < c->E; ++e) {
        rv[e] = c->vinv[c->col_idx[e]];
        rp[e] = c->edge_pos[e];
      }
      auto up = [&](int32_t** d, const int32_t* h, size_t cnt) {
        if (e1 == hipSuccess) e1 = hipMalloc(d, sizeof(int32_t) * std::max<size_t>(cnt, 1));
        if (e1 == hipSuccess && cnt) e1 = hipMemcpy(*d, h, sizeof(int32_t) * cnt, hipMemcpyHostToDevice);
      };
      up(&c->d_row_var, rv.data(), c->E);
      up(&c->d_row_pos, rp.data(), c->E);
      up(&c->d_col_ptr, c->csc_ptr.data(), n + 1);
      up(&c->d_vinv32, c->vinv.data(), n);
    }
    if (e1 == hipSuccess) e1 = hipMalloc(&c->d_row_ptr, sizeof(int32_t) * (m + 1));
    if (e1 == hipSuccess) e1 = hipMemcpy(c->d_row_ptr, c->row_ptr.data(), sizeof(int32_t) * (m + 1), hipMemcpyHostToDevice);
    if (e1 == hipSuccess) e1 = hipMalloc(&c->d_col_idx, sizeof(int32_t) * std::max(1, c->E));
    if (e1 == hipSuccess && c->E) e1 = hipMemcpy(c->d_col_idx, c->col_idx.data(), sizeof(int32_t) * c->E, hipMemcpyHostToDevice);
    if (e1 == hipSuccess && m > 0) {
      std::vector<uint32_t> rtab((size_t)8 * m, 0);
      for (int r = 0; r < m; ++r)
        for (int e = c->row_ptr[r], k = 0; e < c->row_ptr[r + 1] && k < 8; ++e, ++k)
          rtab[(size_t)8 * r + k] = (uint32_t)c->vinv[c->col_idx[e]];
      e1 = hipMalloc(&c->d_wc, sizeof(uint32_t) * m);
      if (e1 == hipSuccess) e1 = hipMemcpy(c->d_wc, c->wc.data(), sizeof(uint32_t) * m, hipMemcpyHostToDevice);
      if (e1 == hipSuccess) e1 = hipMalloc(&c->d_rtab, sizeof(uint32_t) * 8 * m);
      if (e1 == hipSuccess) e1 = hipMemcpy(c->d_rtab, rtab.data(), sizeof(uint32_t) * 8 * m, hipMemcpyHostToDevice);
      if (e1 == hipSuccess) e1 = hipMalloc(&c->d_avar, sizeof(uint32_t) * n);
      if (e1 == hipSuccess) e1 = hipMemcpy(c->d_avar, c->avar.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    }
    if (e1 != hipSuccess) {
      delete c;
      return fail(QLDPC_EHIP, "uploading the graph failed: %s", hipGetErrorString(e1));
    }
  }
  *out = c;
  return QLDPC_OK;
}

static void ws_free(qldpc_code* c) {
  (void)hipFree(c->ws_syn);
  (void)hipFree(c->ws_ehat);
  (void)hipFree(c->ws_iters);
  (void)hipFree(c->ws_flags);
  (void)hipFree(c->ws_post);
  (void)hipHostFree(c->hp_syn);
  (void)hipHostFree(c->hp_ehat);
  (void)hipHostFree(c->hp_iters);
  (void)hipHostFree(c->hp_flags);
  (void)hipHostFree(c->hp_post);
  c->ws_syn = c->ws_ehat = c->hp_syn = c->hp_ehat = nullptr;
  c->ws_iters = c->ws_flags = c->hp_iters = c->hp_flags = nullptr;
  c->ws_post = c->hp_post = nullptr;
  c->ws_cap = 0;
}

extern "C" int qldpc_code_destroy(qldpc_code* code) {
  if (!code) return QLDPC_OK;
  (void)hipFree(code->d_vinv);
  (void)hipFree(code->d_row_ptr);
  (void)hipFree(code->d_col_idx);
  (void)hipFree(code->d_wc);
  (void)hipFree(code->d_rtab);
  (void)hipFree(code->d_avar);
  (void)hipFree(code->d_row_var);
  (void)hipFree(code->d_row_pos);
  (void)hipFree(code->d_col_ptr);
  (void)hipFree(code->d_vinv32);
  ws_free(code);
  if (code->ws_stream) (void)hipStreamDestroy(code->ws_stream);
  delete code;
  return QLDPC_OK;
}

extern "C" int qldpc_code_shape(const qldpc_code* code, int* m, int* n, int* n_edges) {
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (m) *m = code->m;
  if (n) *n = code->n;
  if (n_edges) *n_edges = code->E;
  return QLDPC_OK;
}

// ---------------------------------------------------------------------------
// schedule (layers) + LDS image
// ---------------------------------------------------------------------------
struct LaunchCfg {
  const void* kernel = nullptr;
  int waves = 0, blocks_per_cu = 0, lds = 0, wave_bytes = 0;
  bool lblob = false;  // uses the layer-ordered blob (ms_layered_kernel)
  bool gtab = false;     // ms_flood_kernel: global tables, LDS = wave state only
  bool tlg = false;      // bp_team_lg_kernel: every table global, LDS image = layer pointers
  bool hbm = false;      // the LDS kernels cannot hold this schedule: hbm_tile_kernel (cached)
  int msl_gt = 0;        // ms_layered_kernel<DC, 1> built with QLDPC_MSL_GT: tables left in global memory
  int synl_rows = 0;     // ms_layered_kernel<DC, 0>: layer-ordered syndrome bits per wave (rows)
  uint32_t gen = 0;      // g_opt.gen the configuration was built under
  int team = 0;          // bp_team_kernel: waves per half-shot (one workgroup), 0 = wave kernels
  const char* name = "";  // kernel name as rocprofv3 reports it
  bool ok = false;
};

struct qldpc_schedule {
  const qldpc_code* code = nullptr;
  bool layered = false;
  int n_layers = 0;
  int median_rows = 0;        // rows of the median layer (layered MS lanes-per-check choice)
  int layer_g = 0;            // lanes per check shared by every layer, 0 = chosen per layer
  std::vector<uint8_t> blob;  // LDS image of the graph tables
  // layered MS, uniform degree: layer-ordered tables (ms_layered_kernel)
  std::vector<uint8_t> lblob;
  unsigned char* d_lblob = nullptr;
  int l_off_ltab = 0, l_off_lrow = 0, l_off_lay_ptr = 0, l_off_adj_ptr = 0, l_off_adj_vars = 0,
      l_off_adj_info = 0, l_off_adj_dmax = 0, l_off_vn_chk = 0;
  int off_cn_tab = 0, off_row_ptr = 0, off_vn_ptr = 0, off_vn_chk = 0;
  int off_lay_ptr = 0, off_lay_rows = 0, off_adj_ptr = 0, off_adj_vars = 0, off_chunk_dmax = 0;
  unsigned char* d_blob = nullptr;
  // layered BP teams with every table global (bp_team_lg_kernel): layer
  // pointers (the LDS image), then rows in layer order, their checks, adjacency
  std::vector<uint8_t> lgblob;
  unsigned char* d_lgblob = nullptr;
  int lg_lds_bytes = 0, lg_off_lay_ptr = 0, lg_off_adj_ptr = 0, lg_off_ltab = 0, lg_off_lrow = 0, lg_off_adj = 0;
  // flooding MS, uniform degree: global table image of ms_flood_kernel
  std::vector<uint8_t> fblob;
  unsigned char* d_fblob = nullptr;
  int f_off_tab = 0;
  LaunchCfg cfg[2];           // per algo
  std::mutex mu;
  // HBM-resident kernel (hbm_kernels.hip): 32-bit layer tables and a grow-only
  // slot-major workspace; hbm_ev orders launches that share the workspace
  bool lds_ok = true;         // the LDS kernels' 16-bit layer tables hold this schedule
  bool hbm_lazy = false;      // every row in exactly one layer (no state init pass)
  std::vector<int32_t> h_lay_ptr, h_lay_rows, h_adj_ptr, h_adj_vars, h_fl_var, h_fl_pos;
  int32_t *d_h_lay_ptr = nullptr, *d_h_lay_rows = nullptr, *d_h_adj_ptr = nullptr, *d_h_adj_vars = nullptr,
          *d_h_fl_var = nullptr, *d_h_fl_pos = nullptr;
  void* hbm_ws = nullptr;
  size_t hbm_ws_bytes = 0;
  hipEvent_t hbm_ev = nullptr;
  int hbm_tiles_cap[2] = {0, 0};  // per algo: CUs x resident tiles per CU (queried once)
  // half-shot work-queue counters (ring: concurrent launches on different
  // streams take different slots; each is zeroed on the launch stream)
  static constexpr int kQueueSlots = 64;
  uint32_t* d_queue = nullptr;
  std::atomic<uint32_t> qnext{0};
};

static int align16(int x) { return (x + 15) & ~15; }

// Uniform row degree 7 or 8 with LDS offsets that fit 16 bits -> the
// unrolled kernel instantiation and its pre-scaled table format.
static bool fast_table_ok(const qldpc_code* c) {
  return (c->uniform_deg == 7 || c->uniform_deg == 8) && 8 * c->n < 65536 && 8 * c->E < 65536;
}

template <typename T>
static int put(std::vector<uint8_t>& blob, const std::vector<T>& v) {
  const int off = align16((int)blob.size());
  blob.resize(off + sizeof(T) * v.size());
  if (!v.empty()) memcpy(blob.data() + off, v.data(), sizeof(T) * v.size());
  return off;
}

extern "C" int qldpc_schedule_create(const qldpc_code* code, int n_layers, const int32_t* h_layer_ptr,
                                     const int32_t* h_layer_rows, qldpc_schedule** out) {
  if (!out) return fail(QLDPC_EINVAL, "out is null");
  *out = nullptr;
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (n_layers < 0 || (n_layers > 0 && !h_layer_ptr)) return fail(QLDPC_EINVAL, "bad layer list");
  const int m = code->m, n = code->n;
  std::vector<std::vector<int>> layers(n_layers);
  std::vector<int> seen(m, -1);
  for (int l = 0; l < n_layers; ++l) {
    const int a = h_layer_ptr[l], b = h_layer_ptr[l + 1];
    if (a < 0 || b < a) return fail(QLDPC_EINVAL, "layer_ptr is not non-decreasing at layer %d", l);
    for (int q = a; q < b; ++q) {
      const int r = h_layer_rows[q];
      if (r < 0 || r >= m)
        return fail(QLDPC_ERANGE, "index %d is out of bounds for axis 0 with size %d", r, m);
      if (seen[r] != l) {  // duplicates inside a layer: same Jacobi inputs, same outputs
        seen[r] = l;
        layers[l].push_back(r);
      }
    }
  }
  auto* s = new qldpc_schedule();
  s->code = code;
  s->n_layers = n_layers;
  // One layer holding every row exactly once == flooding (decoders.py:122).
  s->layered = !(n_layers == 1 && (int)layers[0].size() == m);

  // HBM-resident kernel tables (32-bit, every schedule): layer rows, each
  // layer's adjacent variables (ascending), and for the no-init first
  // iteration the first layer that reaches each variable / CSC position
  {
    s->h_lay_ptr.assign(n_layers + 1, 0);
    s->h_adj_ptr.assign(n_layers + 1, 0);
    s->h_fl_var.assign(std::max(n, 1), n_layers);
    s->h_fl_pos.assign(std::max(code->E, 1), n_layers);
    std::vector<int> row_layer(m, -1), mark(n, -1);
    bool part = true;
    for (int l = 0; l < n_layers; ++l) {
      std::vector<int> adj;
      for (int r : layers[l]) {
        s->h_lay_rows.push_back(r);
        if (row_layer[r] >= 0) part = false;          // a row in two layers
        row_layer[r] = l;
        for (int e = code->row_ptr[r]; e < code->row_ptr[r + 1]; ++e) {
          const int v = code->vinv[code->col_idx[e]];
          if (mark[v] != l) {
            mark[v] = l;
            adj.push_back(v);
          }
        }
      }
      std::sort(adj.begin(), adj.end());
      for (int v : adj) {
        s->h_adj_vars.push_back(v);
        s->h_fl_var[v] = std::min(s->h_fl_var[v], l);
      }
      s->h_lay_ptr[l + 1] = (int32_t)s->h_lay_rows.size();
      s->h_adj_ptr[l + 1] = (int32_t)s->h_adj_vars.size();
    }
    for (int r = 0; r < m; ++r) {
      if (row_layer[r] < 0) part = false;             // a row no layer updates
      for (int e = code->row_ptr[r]; e < code->row_ptr[r + 1]; ++e) s->h_fl_pos[code->edge_pos[e]] = row_layer[r];
    }
    s->hbm_lazy = part;
  }
  s->lds_ok = code->lds_ok && s->h_lay_rows.size() <= 65535 && s->h_adj_vars.size() <= 65535;

  if (s->lds_ok) {
  std::vector<uint32_t> cn_tab;
  if (fast_table_ok(code)) {
    // uniform row degree: rows padded to 8 entries, pre-scaled LDS byte offsets
    // (4 * csc position) << 16 | (8 * relabeled variable)
    cn_tab.assign((size_t)8 * m, 0);
    for (int r = 0; r < m; ++r)
      for (int e = code->row_ptr[r], k = 0; e < code->row_ptr[r + 1]; ++e, ++k)
        cn_tab[(size_t)8 * r + k] = ((uint32_t)(4 * code->edge_pos[e]) << 16) |
                                    (uint32_t)(8 * code->vinv[code->col_idx[e]]);
  } else {
    cn_tab.resize(code->E);
    for (int e = 0; e < code->E; ++e)
      cn_tab[e] = ((uint32_t)code->vinv[code->col_idx[e]] << 16) | (uint32_t)code->edge_pos[e];
  }
  std::vector<uint16_t> row_ptr(code->row_ptr.begin(), code->row_ptr.end());
  std::vector<uint32_t> vn_ptr(n);  // csc start | degree << 16
  for (int j = 0; j < n; ++j)
    vn_ptr[j] = (uint32_t)code->csc_ptr[j] | ((uint32_t)(code->csc_ptr[j + 1] - code->csc_ptr[j]) << 16);
  s->off_cn_tab = put(s->blob, cn_tab);
  s->off_row_ptr = put(s->blob, row_ptr);
  s->off_vn_ptr = put(s->blob, vn_ptr);
  std::vector<uint8_t> chunk_dmax((n + 63) / 64, 0);   // VN passes unroll to this (<= 255)
  for (int j = 0; j < n; ++j)
    chunk_dmax[j >> 6] = (uint8_t)std::min(255, std::max<int>(chunk_dmax[j >> 6], code->csc_ptr[j + 1] - code->csc_ptr[j]));
  s->off_chunk_dmax = put(s->blob, chunk_dmax);
  if (s->layered) {
    std::vector<uint16_t> vn_chk(code->E), lay_ptr(n_layers + 1, 0), lay_rows, adj_ptr(n_layers + 1, 0), adj_vars;
    for (int p = 0; p < code->E; ++p) {
      // CSR edge -> its check (row)
      const int e = code->csc_edge[p];
      const int r = (int)(std::upper_bound(code->row_ptr.begin(), code->row_ptr.end(), e) - code->row_ptr.begin()) - 1;
      vn_chk[p] = (uint16_t)r;
    }
    std::vector<int> mark(n, -1);
    for (int l = 0; l < n_layers; ++l) {
      std::vector<int> adj;
      for (int r : layers[l]) {
        lay_rows.push_back((uint16_t)r);
        for (int e = code->row_ptr[r]; e < code->row_ptr[r + 1]; ++e) {
          const int v = code->vinv[code->col_idx[e]];
          if (mark[v] != l) {
            mark[v] = l;
            adj.push_back(v);
          }
        }
      }
      std::sort(adj.begin(), adj.end());
      for (int v : adj) adj_vars.push_back((uint16_t)v);
      if (lay_rows.size() > 65535 || adj_vars.size() > 65535) {
        delete s;
        return fail(QLDPC_EUNSUP, "schedule too large for 16-bit layer tables");
      }
      lay_ptr[l + 1] = (uint16_t)lay_rows.size();
      adj_ptr[l + 1] = (uint16_t)adj_vars.size();
    }
    {
      std::vector<int> rows(n_layers);
      for (int l = 0; l < n_layers; ++l) rows[l] = (int)layers[l].size();
      std::sort(rows.begin(), rows.end());
      s->median_rows = n_layers ? rows[n_layers / 2] : 0;
    }
    s->off_vn_chk = put(s->blob, vn_chk);
    s->off_lay_ptr = put(s->blob, lay_ptr);
    s->off_lay_rows = put(s->blob, lay_rows);
    s->off_adj_ptr = put(s->blob, adj_ptr);
    s->off_adj_vars = put(s->blob, adj_vars);
    if (fast_table_ok(code) && n <= 2048 && code->max_col_deg <= 31) {
      std::vector<uint32_t> ltab((size_t)8 * lay_rows.size(), 0), adj_info(adj_vars.size());
      for (size_t q = 0; q < lay_rows.size(); ++q) {
        const int r = lay_rows[q];
        for (int e = code->row_ptr[r], k = 0; e < code->row_ptr[r + 1]; ++e, ++k)
          ltab[8 * q + k] = ((uint32_t)(4 * code->edge_pos[e]) << 16) | (uint32_t)(4 * code->vinv[code->col_idx[e]]);
      }
      std::vector<uint16_t> adj_dmax(std::max(n_layers, 1), 0);
      for (int l = 0; l < n_layers; ++l) {
        int dmin = 32;
        bool mid = false;                                   // a degree strictly between 3 and dmax
        for (int q = adj_ptr[l]; q < adj_ptr[l + 1]; ++q) {
          const int v = adj_vars[q], d = code->csc_ptr[v + 1] - code->csc_ptr[v];
          adj_info[q] = ((uint32_t)v << 21) | ((uint32_t)d << 16) | (uint32_t)code->csc_ptr[v];
          adj_dmax[l] = (uint16_t)std::max<int>(adj_dmax[l], d);   // d <= 31 here
          dmin = std::min(dmin, d);
        }
        for (int q = adj_ptr[l]; q < adj_ptr[l + 1]; ++q) {
          const int v = adj_vars[q], d = code->csc_ptr[v + 1] - code->csc_ptr[v];
          mid |= d > 3 && d < adj_dmax[l];
        }
        // bit 7: every adjacent variable has degree >= 3 (vn_layer's LO = 3);
        // bit 8: and every degree is 3 or the layer's maximum (vn_layer's TWO)
        if (dmin >= 3 && adj_ptr[l + 1] > adj_ptr[l]) {
          adj_dmax[l] = (uint16_t)(adj_dmax[l] | 0x80);
          if (!mid) adj_dmax[l] = (uint16_t)(adj_dmax[l] | 0x100);
        }
      }
      // bits 5-6: log2 of the layer's lanes per check (ms_layered_kernel<DC, 0>):
      // one lane per check for long layers, a lane group when the layer leaves
      // most of the wave idle (rows <= 8: 8 lanes, <= 16: 4)
      // (two lanes per check on 17-64-row layers measured 5-12 % slower, round 2)
      s->layer_g = -2;
      for (int l = 0; l < n_layers; ++l) {
        const int rows = lay_ptr[l + 1] - lay_ptr[l];
        const int gl = rows <= 8 ? 3 : (rows <= 16 ? 2 : 0);
        adj_dmax[l] = (uint16_t)(adj_dmax[l] | (gl << 5));
        s->layer_g = (s->layer_g == -2 || s->layer_g == (1 << gl)) ? (1 << gl) : 0;
      }
      {
        std::vector<uint32_t> btab((size_t)8 * lay_rows.size(), 0);   // cn_tab words (BP format), layer order
        for (size_t q = 0; q < lay_rows.size(); ++q)
          for (int k = 0; k < 8; ++k) btab[8 * q + k] = cn_tab[(size_t)8 * lay_rows[q] + k];
        s->lg_off_lay_ptr = put(s->lgblob, lay_ptr);
        s->lg_off_adj_ptr = put(s->lgblob, adj_ptr);
        s->lgblob.resize(align16((int)s->lgblob.size() + 1));
        s->lg_lds_bytes = (int)s->lgblob.size();
        s->lg_off_ltab = put(s->lgblob, btab);
        s->lg_off_lrow = put(s->lgblob, lay_rows);
        s->lg_off_adj = put(s->lgblob, adj_info);
        s->lgblob.resize(align16((int)s->lgblob.size() + 1));
      }
      s->l_off_ltab = put(s->lblob, ltab);
      s->l_off_lrow = put(s->lblob, lay_rows);
      s->l_off_lay_ptr = put(s->lblob, lay_ptr);
      s->l_off_adj_ptr = put(s->lblob, adj_ptr);
      s->l_off_adj_info = put(s->lblob, adj_info);
      s->l_off_adj_dmax = put(s->lblob, adj_dmax);
      s->l_off_vn_chk = put(s->lblob, code->avar);   // filter word per relabeled variable
      s->lblob.resize(align16((int)s->lblob.size() + 1));
    }
  }
  if (!s->layered && fast_table_ok(code) && m <= 8 * 64) {
    // ms_flood_kernel's global image: FloodRuns header (runs of equal column
    // degree over the relabeled variables), then per check c = lane + 64 i the
    // words [8c, 8c+8): (4 * csc position) << 16 | (8 * relabeled variable).
    // Pad checks write the pad floats E..E+7 behind c2v and read post[0].
    std::vector<int32_t> hdr(1 + 4 * QLDPC_MAX_RUNS, 0);
    int nr = 0;
    bool ok = true;
    for (int j = 0; j < n;) {
      const int d = code->csc_ptr[j + 1] - code->csc_ptr[j];
      int e = j;
      while (e < n && code->csc_ptr[e + 1] - code->csc_ptr[e] == d) ++e;
      if (nr == QLDPC_MAX_RUNS) { ok = false; break; }
      hdr[1 + nr] = j;                                   // start
      hdr[1 + QLDPC_MAX_RUNS + nr] = e - j;              // count
      hdr[1 + 2 * QLDPC_MAX_RUNS + nr] = d;              // degree
      hdr[1 + 3 * QLDPC_MAX_RUNS + nr] = code->csc_ptr[j];  // csc start
      ++nr;
      j = e;
    }
    hdr[0] = nr;
    if (ok) {
      std::vector<uint32_t> ftab((size_t)8 * 64 * 8, 0);
      for (int r = 0; r < 8 * 64; ++r)
        for (int k = 0; k < 8; ++k) {
          const int e = r < m ? code->row_ptr[r] + k : -1;
          if (r < m && e < code->row_ptr[r + 1])
            ftab[(size_t)8 * r + k] = ((uint32_t)(4 * code->edge_pos[e]) << 16) |
                                      (uint32_t)(8 * code->vinv[code->col_idx[e]]);
          else if (r >= m)
            ftab[(size_t)8 * r + k] = (uint32_t)(4 * (code->E + k)) << 16;
        }
      (void)put(s->fblob, hdr);
      s->f_off_tab = put(s->fblob, ftab);
      s->fblob.resize(align16((int)s->fblob.size() + 1));
    }
  }
  }  // s->lds_ok
  s->blob.resize(align16((int)s->blob.size() + 1));
  if (code->device < 0) {  // no device: keep the host image only
    *out = s;
    return QLDPC_OK;
  }
  hipError_t e1 = hipMalloc(&s->d_blob, s->blob.size());
  if (e1 == hipSuccess) e1 = hipMalloc(&s->d_queue, sizeof(uint32_t) * qldpc_schedule::kQueueSlots);
  if (e1 == hipSuccess) e1 = hipMemcpy(s->d_blob, s->blob.data(), s->blob.size(), hipMemcpyHostToDevice);
  if (e1 == hipSuccess && !s->fblob.empty()) {
    e1 = hipMalloc(&s->d_fblob, s->fblob.size());
    if (e1 == hipSuccess) e1 = hipMemcpy(s->d_fblob, s->fblob.data(), s->fblob.size(), hipMemcpyHostToDevice);
  }
  if (e1 == hipSuccess && !s->lgblob.empty()) {
    e1 = hipMalloc(&s->d_lgblob, s->lgblob.size());
    if (e1 == hipSuccess) e1 = hipMemcpy(s->d_lgblob, s->lgblob.data(), s->lgblob.size(), hipMemcpyHostToDevice);
  }
  if (e1 == hipSuccess && !s->lblob.empty()) {
    e1 = hipMalloc(&s->d_lblob, s->lblob.size());
    if (e1 == hipSuccess) e1 = hipMemcpy(s->d_lblob, s->lblob.data(), s->lblob.size(), hipMemcpyHostToDevice);
  }
  auto up32 = [&](int32_t** d, const std::vector<int32_t>& h) {
    if (e1 == hipSuccess) e1 = hipMalloc(d, sizeof(int32_t) * std::max<size_t>(h.size(), 1));
    if (e1 == hipSuccess && !h.empty()) e1 = hipMemcpy(*d, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice);
  };
  up32(&s->d_h_lay_ptr, s->h_lay_ptr);
  up32(&s->d_h_lay_rows, s->h_lay_rows);
  up32(&s->d_h_adj_ptr, s->h_adj_ptr);
  up32(&s->d_h_adj_vars, s->h_adj_vars);
  up32(&s->d_h_fl_var, s->h_fl_var);
  up32(&s->d_h_fl_pos, s->h_fl_pos);
  if (e1 != hipSuccess) {
    delete s;
    return fail(QLDPC_EHIP, "uploading the schedule failed: %s", hipGetErrorString(e1));
  }
  *out = s;
  return QLDPC_OK;
}

extern "C" int qldpc_schedule_destroy(qldpc_schedule* s) {
  if (!s) return QLDPC_OK;
  (void)hipFree(s->d_blob);
  (void)hipFree(s->d_lblob);
  (void)hipFree(s->d_lgblob);
  (void)hipFree(s->d_fblob);
  (void)hipFree(s->d_queue);
  for (int32_t* d : {s->d_h_lay_ptr, s->d_h_lay_rows, s->d_h_adj_ptr, s->d_h_adj_vars, s->d_h_fl_var, s->d_h_fl_pos})
    (void)hipFree(d);
  (void)hipFree(s->hbm_ws);
  if (s->hbm_ev) (void)hipEventDestroy(s->hbm_ev);
  delete s;
  return QLDPC_OK;
}

extern "C" int qldpc_schedule_release_workspace(qldpc_schedule* s) {
  if (!s) return fail(QLDPC_EINVAL, "schedule is null");
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->hbm_ws) {
    if (s->hbm_ev) HIP_TRY(hipEventSynchronize(s->hbm_ev));   // the last launch that used it is done
    HIP_TRY(hipFree(s->hbm_ws));
    s->hbm_ws = nullptr;
    s->hbm_ws_bytes = 0;
  }
  return QLDPC_OK;
}

// per-wave state slice: post f64[n] | c2v (f32|f64)[E] | syn words | parity words
// (ms_layered_kernel, colsum_f32: the "parity words" slot holds the syndrome
// bits in layer order instead, 2 ceil(synl_rows / 64) words; the lane-group
// instance <DC, 0> only)
static void wave_layout(const qldpc_code* c, bool layered, int algo, int* bytes, int* off_c2v,
                        int* off_synw, int* off_parw, bool colsum_f32 = false, int synl_rows = 0) {
  int off = align16((colsum_f32 ? 4 : 8) * c->n);   // post f64, or ms_layered_kernel's float32 sums
  *off_c2v = off;
  off = align16(off + (algo == QLDPC_ALGO_MS ? 4 : 8) * (c->E + 8));  // +8: VN over-read pad
  const int words = 2 * ((c->m + 63) / 64);
  *off_synw = off;
  if (layered) off = align16(off + 4 * words);
  *off_parw = off;
  if (layered && !colsum_f32) off = align16(off + 4 * words);
  if (layered && colsum_f32) off = align16(off + 4 * 2 * ((synl_rows + 63) / 64));
  *bytes = std::max(off, 16);
}

// bp_team_kernel's slice: post f64[n] | c2v f64[E + 8] | syn words | parity
// words | reduction slots ([2][W] any-flags, [2][2] tickets)
static void team_layout(const qldpc_code* c, int w, int* bytes, int* off_c2v, int* off_synw,
                        int* off_parw, int* off_red) {
  int off = align16(8 * c->n);
  *off_c2v = off;
  off = align16(off + 8 * (c->E + 8));
  const int words = 2 * ((c->m + 63) / 64);
  *off_synw = off;
  off = align16(off + 4 * words);
  *off_parw = off;
  off = align16(off + 4 * words);
  *off_red = off;
  off = align16(off + 4 * (3 * w + 4));   // + [W] filter words (layered stop test)
  *bytes = off;
}

// ms_layered_kernel's LDS image with QLDPC_MSL_GT: the layer-ordered blob
// without its leading row table and its trailing filter words (both read
// from global memory)
static int msl_lds_bytes(const qldpc_schedule* s, int) { return s->l_off_vn_chk - s->l_off_lrow; }

// The launch configuration of (schedule, algo), copied into *out under the
// schedule's lock: a launch keeps its own consistent snapshot even if an
// option change (qldpc_set_option) rebuilds the cached one meanwhile.
static int launch_config(qldpc_schedule* s, int algo, LaunchCfg* out) {
  std::lock_guard<std::mutex> lk(s->mu);
  const uint32_t gen = g_opt.gen.load();
  if (s->cfg[algo].ok && s->cfg[algo].gen == gen) {
    *out = s->cfg[algo];
    return QLDPC_OK;
  }
  LaunchCfg cfg{};                                   // built aside, published whole
  const qldpc_code* c = s->code;
  const int dc = fast_table_ok(c) ? c->uniform_deg : 0;
  cfg.kernel = nullptr;
  int max_waves = QLDPC_MAX_THREADS / 64;
  bool gtab = false;
  if (algo == QLDPC_ALGO_MS && !s->layered && dc > 0 && !s->fblob.empty() && !opt(&Options::flood_generic)) {
    cfg.kernel = qldpc::select_ms_flood_kernel(dc, (c->m + 63) / 64, &cfg.name);
    gtab = cfg.kernel != nullptr;
    if (gtab) max_waves = qldpc::ms_flood_max_waves((c->m + 63) / 64);
  }
  bool use_lblob = false;
  if (!cfg.kernel && algo == QLDPC_ALGO_MS && s->layered && dc > 0 && !s->lblob.empty() &&
      !opt(&Options::layered_generic)) {
    // lanes per check: 8 for one- or two-row layers (serial schedules), else
    // one (interleaved A/B, DESIGN.md §3.2: wider groups lost on 7-60-row layers)
    // lanes per check: one template width when every layer wants the same,
    // else chosen per layer (the runtime switch costs ~5 % where it is not needed)
    int g = s->layer_g > 0 ? s->layer_g : 0;
    if (const int64_t og = opt(&Options::ms_lanes_per_check)) g = (int)og;
    // (several half-shots per wave, ms_layered_grp_kernel, measured 2x slower
    // in round 2: at a fixed LDS budget it halves the waves per CU; removed)
    cfg.kernel = qldpc::select_ms_layered_kernel(dc, g, &cfg.name);
    use_lblob = cfg.kernel != nullptr;
    cfg.msl_gt = use_lblob && g == 1 && s->l_off_ltab == 0 ? QLDPC_MSL_GT : 0;
    cfg.synl_rows = use_lblob && g == 0 ? (int)s->h_lay_rows.size() : 0;
  }
  cfg.lblob = use_lblob;
  cfg.gtab = gtab;
  int team = 0;
  if (!cfg.kernel && algo == QLDPC_ALGO_BP && dc > 0 && !opt(&Options::bp_wave)) {
    // 4 waves per half-shot; 8 when a team's LDS footprint leaves at most 3
    // teams per CU (LP118_2: 67 KB), so a CU still runs >= 16 waves
    int tb = 0, o1, o2, o3, o4;
    team_layout(c, 4, &tb, &o1, &o2, &o3, &o4);
    team = ((int)s->blob.size() + tb > 48 * 1024) ? 8 : 4;
    // Layered: 4-wave teams with every graph table in global memory
    // (bp_team_lg_kernel): LDS holds only the team's state, so a CU runs 4
    // teams (the VGPR cap of 16 team waves) — LP118_2: 2 teams with all-LDS
    // tables, 3 with the row table alone global; the kernel is barrier /
    // latency-bound and BP-L p = 0.1 ran 175 -> 132 -> 108 ms per launch.
    // Schedules without the global image (n > 2048, a column degree > 31) run
    // the all-LDS team kernel; option bp_lg = 0 forces it (tests).
    const bool tlg = s->layered && !s->lgblob.empty() && opt(&Options::bp_lg) != 0;
    if (tlg) team = 4;
    if (const int64_t ow = opt(&Options::bp_team_w)) team = (int)ow;
    if (tlg) {
      cfg.kernel = qldpc::select_bp_team_lg_kernel(dc, team, &cfg.name);
      cfg.tlg = cfg.kernel != nullptr;
    }
    if (!cfg.kernel) cfg.kernel = qldpc::select_bp_team_kernel(s->layered, dc, team, &cfg.name);
    if (!cfg.kernel) team = 0;
  }
  cfg.team = team;
  if (!cfg.kernel) cfg.kernel = qldpc::select_kernel(algo, s->layered, dc, &cfg.name);
  int off_c2v, off_synw, off_parw, off_red;
  wave_layout(c, s->layered, algo, &cfg.wave_bytes, &off_c2v, &off_synw, &off_parw, use_lblob, cfg.synl_rows);
  if (team) team_layout(c, team, &cfg.wave_bytes, &off_c2v, &off_synw, &off_parw, &off_red);
  int max_lds = 0, dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  HIP_TRY(qldpc::configure_kernel(cfg.kernel, max_lds));
  const int blob = gtab ? QLDPC_FLOOD_HDR
                        : cfg.tlg ? s->lg_lds_bytes
                        : cfg.msl_gt ? msl_lds_bytes(s, cfg.msl_gt)
                        : (int)(use_lblob ? s->lblob.size() : s->blob.size());
  // BP kernels stage NumPy's libm tables behind every slice (DecodeArgs::off_libm)
  const int libm = algo == QLDPC_ALGO_BP ? (int)sizeof(qldpc_libm_tab) : 0;
  int best_waves = 0;
  if (team) {  // one team (workgroup of `team` waves) per half-shot
    const int lds = blob + cfg.wave_bytes + libm;
    int nb = 0;
    if (lds <= max_lds)
      HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cfg.kernel, 64 * team, (size_t)lds));
    cfg.waves = team;
    cfg.blocks_per_cu = nb;
    cfg.lds = lds;
    best_waves = nb * team;
    max_waves = 0;  // skip the wave-kernel search below
  }
  for (int w = max_waves; w >= 1; --w) {
    const int lds = blob + w * cfg.wave_bytes + libm;
    if (lds > max_lds) continue;
    int nb = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cfg.kernel, 64 * w, (size_t)lds));
    if (nb * w > best_waves) {
      best_waves = nb * w;
      cfg.waves = w;
      cfg.blocks_per_cu = nb;
      cfg.lds = lds;
    }
  }
  // Tuning overrides (experiments only): options waves_per_wg, wg_per_cu.
  if (const int64_t ow = team ? 0 : opt(&Options::waves_per_wg)) {
    const int w = (int)ow;
    const int lds = blob + w * cfg.wave_bytes + libm;
    int nb = 0;
    if (w >= 1 && w <= max_waves && lds <= max_lds &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cfg.kernel, 64 * w, (size_t)lds) == hipSuccess && nb > 0) {
      cfg.waves = w;
      cfg.blocks_per_cu = nb;
      cfg.lds = lds;
      best_waves = nb * w;
    }
  }
  if (const int64_t ok = opt(&Options::wg_per_cu)) {
    const int k = (int)ok;
    if (k >= 1 && k < cfg.blocks_per_cu) cfg.blocks_per_cu = k;
  }
  // no LDS kernel holds the graph's per-half-shot state and tables: the
  // HBM-resident kernel decodes it (choose_path); decided once per
  // configuration, not per launch
  cfg.hbm = best_waves == 0;
  cfg.ok = true;
  cfg.gen = gen;
  s->cfg[algo] = cfg;
  *out = cfg;
  return QLDPC_OK;
}

// ---------------------------------------------------------------------------
// timing
// ---------------------------------------------------------------------------
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_events;
static double g_total_ms = 0.0;
static int64_t g_launches = 0;

extern "C" int qldpc_timing_enable(int on) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_timing = on != 0;
  return QLDPC_OK;
}

static int drain_events_locked() {
  for (auto& ev : g_events) {
    HIP_TRY(hipEventSynchronize(ev.second));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev.first, ev.second));
    g_total_ms += ms;
    g_launches++;
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  g_events.clear();
  return QLDPC_OK;
}

extern "C" int qldpc_timing_reset(void) {
  std::lock_guard<std::mutex> lk(g_tmu);
  int rc = drain_events_locked();
  g_total_ms = 0.0;
  g_launches = 0;
  return rc;
}

extern "C" int qldpc_timing_read(double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_tmu);
  int rc = drain_events_locked();
  if (total_ms) *total_ms = g_total_ms;
  if (launches) *launches = g_launches;
  return rc;
}

// ---------------------------------------------------------------------------
// decode
// ---------------------------------------------------------------------------
// Which kernel family decodes (schedule, algo): the LDS-resident kernels when
// their tables and per-half-shot state fit, else the HBM-resident kernel
// (hbm_kernels.hip). Option force_hbm takes the HBM kernel for any code
// (tests: the two families agree bit for bit).
static int choose_path(qldpc_schedule* s, int algo, LaunchCfg* cfg, bool* hbm) {
  const qldpc_code* c = s->code;
  *hbm = !s->lds_ok || opt(&Options::force_hbm) != 0 || (algo == QLDPC_ALGO_MS && c->max_row_deg > 32) ||
         (algo == QLDPC_ALGO_BP && c->max_col_deg > 128);
  if (*hbm) return QLDPC_OK;
  const int rc = launch_config(s, algo, cfg);
  if (rc == QLDPC_OK && cfg->hbm) *hbm = true;      // LDS image / state does not fit a CU
  return rc;
}

static void record_timing(hipEvent_t e0, hipEvent_t e1);

// The HBM-resident decode: tiles of 64 half-shot slots, one workgroup each,
// tiles = min(what the batch fills, the workgroups a CU holds at the kernel's
// register use, what a 64 GiB (or half the free memory) workspace holds); the workspace belongs to the schedule and an event
// orders launches that share it.
static int decode_hbm(const qldpc_code* code, qldpc_schedule* s, int algo, const void* d_syn, int syn_format,
                      int64_t batch, double p, int max_iter, double beta, double eps, void* d_ehat,
                      int ehat_format, int32_t* d_iters, double* d_post, int32_t* d_flags, hipStream_t st) {
  const char* name = nullptr;
  const void* kern = qldpc::select_hbm_kernel(algo, code->max_row_deg, &name);
  if (!kern) return fail(QLDPC_EINVAL, "Unrecognized decoder type.");
  const size_t w = algo == QLDPC_ALGO_MS ? 4 : 8;   // message / posterior row element (MS: f32 S)
  const size_t per_tile = ((size_t)code->E * w + (size_t)code->n * w + (size_t)code->m) * 64;
  std::lock_guard<std::mutex> lk(s->mu);
  if (s->hbm_tiles_cap[algo] == 0) {               // resident tiles: queried once per schedule
    int dev = 0, cus = 0, per_cu = 0;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * qldpc::kHbmWaves, 0));
    s->hbm_tiles_cap[algo] = cus * std::max(per_cu, 1);
  }
  int64_t tiles = std::min<int64_t>((batch + 63) / 64, (int64_t)s->hbm_tiles_cap[algo]);
  // the workspace those tiles need; grown (never shrunk: qldpc_schedule_release_workspace
  // frees it) within half of the free device memory, at most 64 GiB
  auto need_of = [&](int64_t t) {
    const size_t op = ((size_t)t * code->E * w * 64 + 255) & ~(size_t)255;
    const size_t os = (op + (size_t)t * code->n * w * 64 + 255) & ~(size_t)255;
    return os + (size_t)t * code->m * 64 + 256;
  };
  if (need_of(tiles) > s->hbm_ws_bytes) {
    size_t free_b = 0, total_b = 0;
    HIP_TRY(hipMemGetInfo(&free_b, &total_b));
    const size_t budget = std::min<size_t>(free_b / 2 + s->hbm_ws_bytes, (size_t)64 << 30);
    tiles = std::min<int64_t>(tiles, (int64_t)(budget / per_tile));
  }
  if (tiles < 1) return fail(QLDPC_EUNSUP, "HBM decode needs %zu B per 64-slot tile: device memory too small", per_tile);
  const size_t off_post = ((size_t)tiles * code->E * w * 64 + 255) & ~(size_t)255;
  const size_t off_syn = (off_post + (size_t)tiles * code->n * w * 64 + 255) & ~(size_t)255;
  const size_t need = off_syn + (size_t)tiles * code->m * 64 + 256;
  if (!s->hbm_ev) HIP_TRY(hipEventCreateWithFlags(&s->hbm_ev, hipEventDisableTiming));
  if (need > s->hbm_ws_bytes) {
    if (s->hbm_ws) {
      HIP_TRY(hipEventSynchronize(s->hbm_ev));      // last launch done with the old workspace
      HIP_TRY(hipFree(s->hbm_ws));
      s->hbm_ws = nullptr;
      s->hbm_ws_bytes = 0;
    }
    HIP_TRY(hipMalloc(&s->hbm_ws, need));
    s->hbm_ws_bytes = need;
  }
  HIP_TRY(hipStreamWaitEvent(st, s->hbm_ev, 0));    // a launch on another stream may still use it
  qldpc::HbmArgs a{};
  a.row_ptr = code->d_row_ptr;
  a.row_var = code->d_row_var;
  a.row_pos = code->d_row_pos;
  a.col_ptr = code->d_col_ptr;
  a.vinv = code->d_vinv32;
  a.wc = code->d_wc;
  a.avar = code->d_avar;
  a.filt_all = code->filt_all;
  a.lay_ptr = s->d_h_lay_ptr;
  a.lay_rows = s->d_h_lay_rows;
  a.adj_ptr = s->d_h_adj_ptr;
  a.adj_vars = s->d_h_adj_vars;
  a.n_layers = s->n_layers;
  a.m = code->m;
  a.n = code->n;
  a.E = code->E;
  a.c2v = s->hbm_ws;
  a.post = (char*)s->hbm_ws + off_post;
  a.synT = (uint8_t*)s->hbm_ws + off_syn;
  a.syn = (const uint8_t*)d_syn;
  a.ehat = (uint8_t*)d_ehat;
  a.iters = d_iters;
  a.out_post = d_post;
  a.flags = d_flags;
  a.syn_bits = syn_format == QLDPC_FMT_BITS;
  a.eh_bits = ehat_format == QLDPC_FMT_BITS;
  a.wm = (code->m + 63) / 64;
  a.wn = (code->n + 63) / 64;
  a.batch = batch;
  a.queue = s->d_queue + (s->qnext.fetch_add(1) % qldpc_schedule::kQueueSlots);
  a.L = qldpc_prior_llr(p, eps);                    // np.log prior (decoders.py:147, :232)
  a.L32 = (float)a.L;
  a.beta = beta;
  a.eps = eps;
  a.max_iter = max_iter;
  HIP_TRY(hipMemsetAsync(a.queue, 0, sizeof(uint32_t), st));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  bool timed;
  {
    std::lock_guard<std::mutex> tk(g_tmu);
    timed = g_timing;
  }
  if (timed) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, st));
  }
  HIP_TRY(qldpc::launch_hbm(kern, a, (int)tiles, s->d_h_fl_var, s->d_h_fl_pos, s->hbm_lazy ? 1 : 0, st));
  if (timed) {
    HIP_TRY(hipEventRecord(e1, st));
    record_timing(e0, e1);
  }
  HIP_TRY(hipEventRecord(s->hbm_ev, st));
  return QLDPC_OK;
}

static void record_timing(hipEvent_t e0, hipEvent_t e1) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_events.emplace_back(e0, e1);
}

extern "C" int qldpc_decode_device(const qldpc_code* code, const qldpc_schedule* sched_c, int algo,
                                   const uint8_t* d_syn, int64_t batch, double p, int max_iter,
                                   double beta, double eps, uint8_t* d_ehat, int32_t* d_iters,
                                   double* d_post, int32_t* d_flags, void* stream) {
  return qldpc_decode_device_ex(code, sched_c, algo, d_syn, QLDPC_FMT_BYTES, batch, p, max_iter, beta, eps, d_ehat,
                                QLDPC_FMT_BYTES, d_iters, d_post, d_flags, stream);
}

// The BP check node's saturated value (decoder_kernels.hip, cn_bp_word): at
// |th2| = 1 the reference clips th2 to +-(1 - eps) (decoders.py:256-258), so
// c2v = +-2 atanh(1 - eps) — computed here by the restated SVML atanh the
// kernels and the oracle share (include/qldpc_libm.h), the same expression
// as the full path; not finite (eps <= 0) turns the fast path off.
static void bp_saturation(double eps, double* csat, uint32_t* sat_hi) {
  double th2 = 1.0;
  th2 = (std::fabs(th2) >= 1.0 - eps) ? std::copysign(std::fabs(th2) - eps, th2) : th2;
  const double v = 2.0 * qldpc_atanh(th2);
  const bool on = std::isfinite(v);
  *csat = on ? v : 0.0;
  *sat_hi = on ? 0x40338000u : 0x7ff00000u;            // |x| >= 19.5 (high word, sign cleared)
}

extern "C" int qldpc_decode_device_ex(const qldpc_code* code, const qldpc_schedule* sched_c, int algo,
                                      const void* d_syn, int syn_format, int64_t batch, double p, int max_iter,
                                      double beta, double eps, void* d_ehat, int ehat_format, int32_t* d_iters,
                                      double* d_post, int32_t* d_flags, void* stream) {
  auto* sched = const_cast<qldpc_schedule*>(sched_c);
  if ((syn_format != QLDPC_FMT_BYTES && syn_format != QLDPC_FMT_BITS) ||
      (ehat_format != QLDPC_FMT_BYTES && ehat_format != QLDPC_FMT_BITS))
    return fail(QLDPC_EINVAL, "unknown syndrome / estimate format");
  if (!code || !sched) return fail(QLDPC_EINVAL, "code/schedule is null");
  if (sched->code != code) return fail(QLDPC_EINVAL, "schedule was built for a different code");
  if (algo != QLDPC_ALGO_MS && algo != QLDPC_ALGO_BP) return fail(QLDPC_EINVAL, "Unrecognized decoder type.");
  if (batch < 0) return fail(QLDPC_EINVAL, "negative batch");
  if (max_iter < 1) return fail(QLDPC_EINVAL, "max_iter must be >= 1 (the reference leaves e_hat unbound)");
  if (batch == 0) return QLDPC_OK;
  if (!d_syn || !d_ehat || !d_iters) return fail(QLDPC_EINVAL, "null device buffer");
  if (code->device < 0 || !sched->d_blob) return fail(QLDPC_EHIP, "no HIP device was visible when the code/schedule was created");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != code->device) return fail(QLDPC_EINVAL, "code lives on device %d, current device is %d", code->device, dev);
  LaunchCfg cfgv;
  LaunchCfg* cfg = &cfgv;
  bool hbm = false;
  int rc = choose_path(sched, algo, cfg, &hbm);
  if (rc) return rc;
  if (hbm)
    return decode_hbm(code, sched, algo, d_syn, syn_format, batch, p, max_iter, beta, eps, d_ehat, ehat_format,
                      d_iters, d_post, d_flags, (hipStream_t)stream);

  DecodeArgs a{};
  a.blob = sched->d_blob;
  a.blob_bytes = (int)sched->blob.size();
  a.off_cn_tab = sched->off_cn_tab;
  a.off_row_ptr = sched->off_row_ptr;
  a.off_vn_ptr = sched->off_vn_ptr;
  a.off_vn_chk = sched->off_vn_chk;
  a.off_lay_ptr = sched->off_lay_ptr;
  a.off_lay_rows = sched->off_lay_rows;
  a.off_adj_ptr = sched->off_adj_ptr;
  a.off_adj_vars = sched->off_adj_vars;
  a.off_chunk_dmax = sched->off_chunk_dmax;
  wave_layout(code, sched->layered, algo, &a.wave_bytes, &a.off_c2v, &a.off_synw, &a.off_parw, cfg->lblob,
              cfg->synl_rows);
  if (cfg->lblob) {  // ms_layered_kernel's blob: field mapping documented in the kernel
    a.blob = sched->d_lblob;
    a.blob_bytes = (int)sched->lblob.size();
    a.off_cn_tab = sched->l_off_ltab;
    a.off_lay_rows = sched->l_off_lrow;
    a.off_lay_ptr = sched->l_off_lay_ptr;
    a.off_adj_ptr = sched->l_off_adj_ptr;
    a.off_adj_vars = sched->l_off_adj_vars;
    a.off_row_ptr = sched->l_off_adj_info;
    a.off_chunk_dmax = sched->l_off_adj_dmax;
    a.off_vn_chk = sched->l_off_vn_chk;
    if (cfg->msl_gt) {  // row table (offset 0) and filter words (last) stay global
      a.lds_skip = sched->l_off_lrow;
      a.blob_bytes = msl_lds_bytes(sched, cfg->msl_gt);
    }
  }
  if (cfg->team) team_layout(code, cfg->team, &a.wave_bytes, &a.off_c2v, &a.off_synw, &a.off_parw, &a.off_red);
  if (cfg->tlg) {  // bp_team_lg_kernel: layer pointers in LDS, every table global
    a.blob = sched->d_lgblob;
    a.blob_bytes = sched->lg_lds_bytes;
    a.off_lay_ptr = sched->lg_off_lay_ptr;
    a.off_adj_ptr = sched->lg_off_adj_ptr;
    a.off_cn_tab = sched->lg_off_ltab;
    a.off_lay_rows = sched->lg_off_lrow;
    a.off_row_ptr = sched->lg_off_adj;
  }
  if (cfg->gtab) {  // global tables; the LDS holds wave state only
    a.blob = sched->d_fblob;
    a.blob_bytes = 0;
    a.off_cn_tab = sched->f_off_tab;
  }
  a.m = code->m;
  a.n = code->n;
  a.E = code->E;
  a.n_layers = sched->n_layers;
  a.vinv = code->d_vinv;
  a.syn = (const uint8_t*)d_syn;
  a.ehat = (uint8_t*)d_ehat;
  a.syn_bits = syn_format == QLDPC_FMT_BITS;
  a.eh_bits = ehat_format == QLDPC_FMT_BITS;
  a.wm = (code->m + 63) / 64;
  a.wn = (code->n + 63) / 64;
  a.iters = d_iters;
  a.post = d_post;
  a.flags = d_flags;
  a.batch = batch;
  // L_ch = np.log((1 - p) / max(p, eps))   (decoders.py:147, :232), with
  // NumPy's own log (SVML log8_ha, include/qldpc_libm.h): glibc's differs in
  // the last bit for ~0.2 % of priors
  a.L = qldpc_prior_llr(p, eps);
  a.off_libm = algo == QLDPC_ALGO_BP ? cfg->lds - (int)sizeof(qldpc_libm_tab) : 0;
  a.L32 = (float)a.L;
  a.beta = beta;
  a.eps = eps;
  bp_saturation(eps, &a.bp_csat, &a.bp_sat_hi);
  a.max_iter = max_iter;
  a.wc = code->d_wc;
  a.rtab = code->d_rtab;
  a.avar = code->d_avar;
  a.filt_all = code->filt_all;
  {
    // (L + (double)S < 0) == (S < hd_thresh) for every float S: the float at
    // or below -L, nudged up one step when -L is not a float
    const double t = -a.L;
    float f = (float)t;
    if ((double)f > t) f = std::nextafter(f, -INFINITY);
    a.hd_thresh = ((double)f == t) ? f : std::nextafter(f, INFINITY);
  }

  a.queue = nullptr;
  if (!opt(&Options::static_sched)) {
    a.queue = sched->d_queue + (sched->qnext.fetch_add(1) % qldpc_schedule::kQueueSlots);
  }
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t per_block = cfg->team ? 1 : (int64_t)cfg->waves;
  const int64_t need = (batch + per_block - 1) / per_block;
  const int64_t resident = (int64_t)cfg->blocks_per_cu * cus;
  const int grid = (int)std::max<int64_t>(1, std::min(need, resident));
  hipStream_t st = (hipStream_t)stream;

  if (a.queue) HIP_TRY(hipMemsetAsync(a.queue, 0, sizeof(uint32_t), st));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  bool timed;
  {
    std::lock_guard<std::mutex> lk(g_tmu);
    timed = g_timing;
  }
  if (timed) {
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, st));
  }
  HIP_TRY(qldpc::launch_decode(cfg->kernel, a, grid, 64 * cfg->waves, cfg->lds, st));
  if (timed) {
    HIP_TRY(hipEventRecord(e1, st));
    std::lock_guard<std::mutex> lk(g_tmu);
    g_events.emplace_back(e0, e1);
  }
  return QLDPC_OK;
}

extern "C" int qldpc_decode_kernel_name(const qldpc_code* code, const qldpc_schedule* sched_c, int algo,
                                        char* buf, int len) {
  auto* sched = const_cast<qldpc_schedule*>(sched_c);
  if (!code || !sched || !buf || len <= 0) return fail(QLDPC_EINVAL, "null argument");
  if (algo != QLDPC_ALGO_MS && algo != QLDPC_ALGO_BP) return fail(QLDPC_EINVAL, "Unrecognized decoder type.");
  if (code->device < 0 || !sched->d_blob) return fail(QLDPC_EHIP, "no HIP device was visible when the code/schedule was created");
  LaunchCfg cfgv;
  LaunchCfg* cfg = &cfgv;
  bool hbm = false;
  int rc = choose_path(sched, algo, cfg, &hbm);
  if (rc) return rc;
  const char* hname = nullptr;
  if (hbm) (void)qldpc::select_hbm_kernel(algo, code->max_row_deg, &hname);
  snprintf(buf, (size_t)len, "%s", hbm ? hname : cfg->name);
  return QLDPC_OK;
}

extern "C" int qldpc_decode_launch_info(const qldpc_code* code, const qldpc_schedule* sched_c, int algo,
                                        int* waves_per_wg, int* wg_per_cu, int* lds_bytes) {
  auto* sched = const_cast<qldpc_schedule*>(sched_c);
  if (!code || !sched || !waves_per_wg || !wg_per_cu || !lds_bytes) return fail(QLDPC_EINVAL, "null argument");
  if (algo != QLDPC_ALGO_MS && algo != QLDPC_ALGO_BP) return fail(QLDPC_EINVAL, "Unrecognized decoder type.");
  if (code->device < 0 || !sched->d_blob) return fail(QLDPC_EHIP, "no HIP device was visible when the code/schedule was created");
  LaunchCfg cfgv;
  LaunchCfg* cfg = &cfgv;
  bool hbm = false;
  int rc = choose_path(sched, algo, cfg, &hbm);
  if (rc) return rc;
  *waves_per_wg = hbm ? 0 : cfg->waves;
  *wg_per_cu = hbm ? 0 : cfg->blocks_per_cu;
  *lds_bytes = hbm ? 0 : cfg->lds;
  return QLDPC_OK;
}

extern "C" int qldpc_decode_host(const qldpc_code* code_c, const qldpc_schedule* sched, int algo,
                                 const uint8_t* h_syn, int64_t batch, double p, int max_iter,
                                 double beta, double eps, uint8_t* h_ehat, int32_t* h_iters,
                                 double* h_post, int32_t* h_flags) {
  auto* code = const_cast<qldpc_code*>(code_c);
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (batch < 0) return fail(QLDPC_EINVAL, "negative batch");
  if (batch == 0) return QLDPC_OK;
  if (!h_syn || !h_ehat || !h_iters) return fail(QLDPC_EINVAL, "null host buffer");
  if (code->device < 0) return fail(QLDPC_EHIP, "no HIP device was visible when the code was created");
  std::lock_guard<std::mutex> lk(code->ws_mu);
  const int m = code->m, n = code->n;
  if (!code->ws_stream) HIP_TRY(hipStreamCreateWithFlags(&code->ws_stream, hipStreamNonBlocking));
  if (batch > code->ws_cap) {
    ws_free(code);
    const int64_t cap = std::max<int64_t>(batch, 64);
    HIP_TRY(hipMalloc(&code->ws_syn, std::max<int64_t>(1, cap * m)));
    HIP_TRY(hipMalloc(&code->ws_ehat, std::max<int64_t>(1, cap * n)));
    HIP_TRY(hipMalloc(&code->ws_iters, sizeof(int32_t) * cap));
    HIP_TRY(hipMalloc(&code->ws_flags, sizeof(int32_t) * cap));
    HIP_TRY(hipMalloc(&code->ws_post, sizeof(double) * std::max<int64_t>(1, cap * n)));
    HIP_TRY(hipHostMalloc(&code->hp_syn, std::max<int64_t>(1, cap * m)));
    HIP_TRY(hipHostMalloc(&code->hp_ehat, std::max<int64_t>(1, cap * n)));
    HIP_TRY(hipHostMalloc(&code->hp_iters, sizeof(int32_t) * cap));
    HIP_TRY(hipHostMalloc(&code->hp_flags, sizeof(int32_t) * cap));
    HIP_TRY(hipHostMalloc(&code->hp_post, sizeof(double) * std::max<int64_t>(1, cap * n)));
    code->ws_cap = cap;
  }
  hipStream_t st = code->ws_stream;
  if (batch * m) {
    memcpy(code->hp_syn, h_syn, batch * m);
    HIP_TRY(hipMemcpyAsync(code->ws_syn, code->hp_syn, batch * m, hipMemcpyHostToDevice, st));
  }
  int rc = qldpc_decode_device(code, sched, algo, code->ws_syn, batch, p, max_iter, beta, eps,
                               code->ws_ehat, code->ws_iters, h_post ? code->ws_post : nullptr,
                               code->ws_flags, st);
  if (rc) return rc;
  if (batch * n) HIP_TRY(hipMemcpyAsync(code->hp_ehat, code->ws_ehat, batch * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(code->hp_iters, code->ws_iters, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(code->hp_flags, code->ws_flags, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, st));
  if (h_post && batch * n)
    HIP_TRY(hipMemcpyAsync(code->hp_post, code->ws_post, sizeof(double) * batch * n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));                  // this stream only
  if (batch * n) memcpy(h_ehat, code->hp_ehat, batch * n);
  memcpy(h_iters, code->hp_iters, sizeof(int32_t) * batch);
  if (h_flags) memcpy(h_flags, code->hp_flags, sizeof(int32_t) * batch);
  if (h_post && batch * n) memcpy(h_post, code->hp_post, sizeof(double) * batch * n);
  return QLDPC_OK;
}

// ---------------------------------------------------------------------------
// GF(2) rank of H by XOR-basis insertion of its columns (gf2math.rank,
// gf2math.py:91-135 — rank is basis independent).
// ---------------------------------------------------------------------------
struct Gf2Basis {
  int mw;
  std::vector<uint64_t> vec;  // [m][mw], slot b holds a vector whose lowest set bit is b
  std::vector<char> has;
  Gf2Basis(int m, int mw_) : mw(mw_), vec((size_t)std::max(m, 1) * std::max(mw_, 1), 0), has(std::max(m, 1), 0) {}
  // returns true if x (modified) was independent and got inserted
  bool insert(uint64_t* x) {
    for (int w = 0; w < mw; ++w) {
      while (x[w]) {
        const int b = w * 64 + __builtin_ctzll(x[w]);
        if (!has[b]) {
          memcpy(&vec[(size_t)b * mw], x, sizeof(uint64_t) * mw);
          has[b] = 1;
          return true;
        }
        const uint64_t* v = &vec[(size_t)b * mw];
        for (int k = w; k < mw; ++k) x[k] ^= v[k];
      }
    }
    return false;
  }
};

static int gf2_rank_cols(const std::vector<uint64_t>& cols, int n, int mw) {
  if (mw == 0) return 0;
  Gf2Basis B(mw * 64, mw);
  std::vector<uint64_t> x(mw);
  int r = 0;
  for (int j = 0; j < n; ++j) {
    memcpy(x.data(), &cols[(size_t)j * mw], sizeof(uint64_t) * mw);
    r += B.insert(x.data());
  }
  return r;
}

// OSD's column bit-vectors and rank(H), built once on first OSD use
static void code_osd_prep(const qldpc_code* c) {
  std::call_once(c->osd_once, [c] {
    c->col_bits.assign((size_t)c->n * std::max(c->mw, 1), 0);
    for (int r = 0; r < c->m; ++r)
      for (int e = c->row_ptr[r]; e < c->row_ptr[r + 1]; ++e)
        c->col_bits[(size_t)c->col_idx[e] * c->mw + (r >> 6)] |= 1ull << (r & 63);
    c->rank = gf2_rank_cols(c->col_bits, c->n, c->mw);
  });
}

// Order of iteration of CPython's `set(range(n)) - set(J)` (the reference's
// infoSet, decoders.py:344): returns its first element. Emulates
// setobject.c (set_difference -> set_add_entry / set_table_resize /
// set_insert_clean; LINEAR_PROBES 9, PERTURB_SHIFT 5) for small-int keys
// (hash(i) == i). Verified against the interpreter in tests.
static int cpython_setdiff_first(int n, const std::vector<char>& inJ, int nJ) {
  if (nJ == n) return -1;
  if ((n >> 2) > nJ) {
    // set_copy_and_difference: a copy of set(range(n)) (ascending slots)
    for (int i = 0; i < n; ++i)
      if (!inJ[i]) return i;
    return -1;
  }
  size_t mask = 7;
  std::vector<int64_t> table(8, -1);
  size_t fill = 0, used = 0;
  auto insert_clean = [](std::vector<int64_t>& t, size_t msk, int64_t key) {
    size_t perturb = (size_t)key, i = (size_t)key & msk;
    while (true) {
      if (t[i] < 0) { t[i] = key; return; }
      if (i + 9 <= msk) {
        for (int j = 0; j < 9; ++j) {
          ++i;
          if (t[i] < 0) { t[i] = key; return; }
        }
      }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & msk;
    }
  };
  for (int key = 0; key < n; ++key) {
    if (inJ[key]) continue;
    // set_add_entry (new key, no dummies)
    size_t perturb = (size_t)key, i = (size_t)key & mask;
    while (true) {
      size_t probes = (i + 9 <= mask) ? 9 : 0;
      size_t k = i;
      bool placed = false;
      while (true) {
        if (table[k] < 0) {
          table[k] = key;
          placed = true;
          break;
        }
        if (probes-- == 0) break;
        ++k;
      }
      if (placed) break;
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
    ++fill;
    ++used;
    if (fill * 5 >= mask * 3) {
      const size_t minused = used > 50000 ? used * 2 : used * 4;
      size_t newsize = 8;
      while (newsize <= minused) newsize <<= 1;
      std::vector<int64_t> nt(newsize, -1);
      for (size_t s2 = 0; s2 <= mask; ++s2)
        if (table[s2] >= 0) insert_clean(nt, newsize - 1, table[s2]);
      table.swap(nt);
      mask = newsize - 1;
    }
  }
  for (size_t s2 = 0; s2 <= mask; ++s2)
    if (table[s2] >= 0) return (int)table[s2];
  return -1;
}

extern "C" int qldpc_cpython_setdiff_first(int n, const int32_t* J, int nJ) {
  std::vector<char> inJ(std::max(n, 1), 0);
  int cnt = 0;
  for (int k = 0; k < nJ; ++k)
    if (J[k] >= 0 && J[k] < n && !inJ[J[k]]) inJ[J[k]] = 1, ++cnt;
  return cpython_setdiff_first(n, inJ, cnt);
}

// ---------------------------------------------------------------------------
// OSD (decoders.py:299-370), given the caller's reliability order `perm`
// (np.argsort of decoders.py:320-325 — NumPy's own exp/argsort decide ties).
// ---------------------------------------------------------------------------
static int osd_one(const qldpc_code* c, const uint8_t* syn, const int32_t* perm, int order, uint8_t* ehat,
                   int32_t* J_out, int32_t* J_size, int first_info_index) {
  const int m = c->m, n = c->n, mw = c->mw;
  if (n == 0) return QLDPC_OK;
  code_osd_prep(c);
  // (1) least reliable basis J (decoders.py:329-342): index 0 unconditionally,
  //     then every column (in perm order) that raises the rank, until rank(H).
  Gf2Basis B(std::max(mw * 64, 1), mw);
  std::vector<uint64_t> x(std::max(mw, 1));
  std::vector<int> J;
  std::vector<char> inJ(n, 0);
  auto col = [&](int i) { return &c->col_bits[(size_t)perm[i] * mw]; };
  if (mw) memcpy(x.data(), col(0), sizeof(uint64_t) * mw);
  int rank = mw ? (int)B.insert(x.data()) : 0;
  J.push_back(0);
  inJ[0] = 1;
  if (rank >= c->rank)
    return fail(QLDPC_ERANGE, "index %d is out of bounds for axis 1 with size %d", n, n);  // reference IndexError
  int next = 1;
  while (true) {
    if (next >= n) return fail(QLDPC_ERANGE, "index %d is out of bounds for axis 1 with size %d", n, n);
    memcpy(x.data(), col(next), sizeof(uint64_t) * mw);
    if (B.insert(x.data())) {
      J.push_back(next);
      inJ[next] = 1;
      if (++rank >= c->rank) break;
    }
    ++next;
  }
  const int nJ = (int)J.size();
  if (J_out)
    for (int k = 0; k < nJ; ++k) J_out[k] = J[k];
  if (J_size) *J_size = nJ;
  // (2) e_hat_perm = e_hat[perm]; order-k loop with aliasing:
  //     the cumulative flip is I[0] for order 1 and nothing otherwise.
  std::vector<uint8_t> ep(n);
  for (int i = 0; i < n; ++i) ep[i] = ehat[perm[i]] & 1;
  if (order == 1 && nJ < n) {
    int i0 = first_info_index >= 0 ? first_info_index : cpython_setdiff_first(n, inJ, nJ);
    if (i0 < 0 || i0 >= n || inJ[i0]) return fail(QLDPC_EINVAL, "bad first_info_index %d", i0);
    ep[i0] ^= 1;
  }
  // (3) sJ = (syndrome + Hp[:, I] @ e_I) % 2
  std::vector<uint64_t> sJ(std::max(mw, 1), 0);
  for (int r = 0; r < m; ++r)
    if (syn[r] & 1) sJ[r >> 6] |= 1ull << (r & 63);
  for (int i = 0; i < n; ++i)
    if (!inJ[i] && ep[i]) {
      const uint64_t* cb = col(i);
      for (int w = 0; w < mw; ++w) sJ[w] ^= cb[w];
    }
  // (4) (T @ sJ) % 2 with T from REF(Hp[:, J], reduced=True) (gf2math.py:139-187):
  //     the same row operations applied to sJ as an augmented column.
  const int rw = (nJ + 63) / 64;
  std::vector<uint64_t> rows((size_t)m * rw, 0);
  for (int k = 0; k < nJ; ++k) {
    const uint64_t* cb = col(J[k]);
    for (int w = 0; w < mw; ++w) {
      uint64_t bits = cb[w];
      while (bits) {
        const int r = w * 64 + __builtin_ctzll(bits);
        bits &= bits - 1;
        rows[(size_t)r * rw + (k >> 6)] |= 1ull << (k & 63);
      }
    }
  }
  std::vector<uint8_t> s(m);
  for (int r = 0; r < m; ++r) s[r] = (sJ[r >> 6] >> (r & 63)) & 1;
  auto bit = [&](int r, int k) { return (rows[(size_t)r * rw + (k >> 6)] >> (k & 63)) & 1; };
  auto xor_row = [&](int dst, int src) {
    for (int w = 0; w < rw; ++w) rows[(size_t)dst * rw + w] ^= rows[(size_t)src * rw + w];
    s[dst] ^= s[src];
  };
  int xr = 0;
  for (int k = 0; k < nJ && m > 0; ++k) {
    int r = xr;
    while (r < m && !bit(r, k)) ++r;
    if (r == m) continue;
    if (r != xr) {
      for (int w = 0; w < rw; ++w) std::swap(rows[(size_t)xr * rw + w], rows[(size_t)r * rw + w]);
      std::swap(s[xr], s[r]);
    }
    for (int t = r + 1; t < m; ++t)
      if (bit(t, k)) xor_row(t, xr);
    for (int t = 0; t < xr; ++t)
      if (bit(t, k)) xor_row(t, xr);
    if (++xr >= m) break;
  }
  for (int k = 0; k < nJ; ++k) ep[J[k]] = k < m ? s[k] : 0;
  for (int i = 0; i < n; ++i) ehat[perm[i]] = ep[i];  // e_hat[perm] = ... (:368)
  return QLDPC_OK;
}

extern "C" int qldpc_osd_decode(const qldpc_code* code, const uint8_t* h_syn, const int32_t* h_perm, int order,
                                uint8_t* h_ehat, int32_t* h_J, int32_t* h_J_size, int first_info_index) {
  if (!code || !h_perm || !h_ehat || (!h_syn && code->m)) return fail(QLDPC_EINVAL, "null argument");
  std::vector<char> seen(code->n, 0);
  for (int i = 0; i < code->n; ++i) {
    if (h_perm[i] < 0 || h_perm[i] >= code->n || seen[h_perm[i]]) return fail(QLDPC_EINVAL, "perm is not a permutation");
    seen[h_perm[i]] = 1;
  }
  return osd_one(code, h_syn, h_perm, order, h_ehat, h_J, h_J_size, first_info_index);
}

int qldpc_host_thread_budget();                         // np_order.cpp

extern "C" int qldpc_osd_decode_batch(const qldpc_code* code, int64_t count, const uint8_t* h_syn,
                                      const int32_t* h_perm, int order, uint8_t* h_ehat, int nthreads) {
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (count <= 0) return QLDPC_OK;
  if (nthreads <= 0) nthreads = qldpc_host_thread_budget();
  nthreads = (int)std::min<int64_t>(nthreads, count);
  const int m = code->m, n = code->n;
  std::atomic<int64_t> next{0};
  std::atomic<int> rc{QLDPC_OK};
  std::string err;
  std::mutex emu;
  auto worker = [&]() {
    while (true) {
      const int64_t b = next.fetch_add(1);
      if (b >= count || rc.load() != QLDPC_OK) return;
      const int r = qldpc_osd_decode(code, h_syn + b * m, h_perm + b * n, order, h_ehat + b * n,
                                     nullptr, nullptr, -1);
      if (r != QLDPC_OK) {
        std::lock_guard<std::mutex> lk(emu);
        if (rc.load() == QLDPC_OK) err = g_err;
        rc = r;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  if (rc.load() != QLDPC_OK) g_err = err;
  return rc.load();
}

// ---------------------------------------------------------------------------
// GPU OSD (osd_kernels.hip): one workgroup per shot.
// ---------------------------------------------------------------------------
static int setdiff_table_ints(int n) {
  // largest (new table + old table) CPython's set reaches inserting n keys
  size_t mask = 7, fill = 0, best = 16;
  for (int used = 1; used <= n; ++used) {
    ++fill;
    if (fill * 5 >= mask * 3) {
      const size_t minused = used > 50000 ? (size_t)used * 2 : (size_t)used * 4;
      size_t ns = 8;
      while (ns <= minused) ns <<= 1;
      best = std::max(best, ns + mask + 1);
      mask = ns - 1;
    }
  }
  return (int)best;
}

static int osd_device_impl(const qldpc_code* code, int64_t count, const uint8_t* d_syn, const int32_t* d_perm,
                           const int32_t* d_tiepos, const double* d_post, int order, uint8_t* d_ehat,
                           int32_t* d_status, void* stream);
struct SpillCfg {
  double* post = nullptr;
  int32_t* idx = nullptr;
  int32_t* count = nullptr;
  int64_t cap = 0;
};
static thread_local SpillCfg g_spill;               // set by qldpc_osd_device_ordered_ex for one call

extern "C" int qldpc_osd_device(const qldpc_code* code, int64_t count, const uint8_t* d_syn,
                                const int32_t* d_perm, int order, uint8_t* d_ehat, int32_t* d_status,
                                void* stream) {
  return osd_device_impl(code, count, d_syn, d_perm, nullptr, nullptr, order, d_ehat, d_status, stream);
}

extern "C" int qldpc_osd_order_device(const qldpc_code* code, int64_t count, const double* d_post,
                                      int32_t* d_perm, int32_t* d_tiepos, void* stream) {
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (count < 0) return fail(QLDPC_EINVAL, "negative count");
  if (count == 0) return QLDPC_OK;
  if (code->device < 0) return fail(QLDPC_EHIP, "no HIP device was visible when the code was created");
  if (!d_post || !d_perm || !d_tiepos) return fail(QLDPC_EINVAL, "null device buffer");
  const int n = code->n;
  if (n < 1 || n > 2048) return fail(QLDPC_EUNSUP, "the device reliability order supports 1 <= n <= 2048 (got %d)", n);
  qldpc::OrderArgs a{};
  a.post = d_post;
  a.perm = d_perm;
  a.tiepos = d_tiepos;
  a.n = n;
  HIP_TRY(qldpc::launch_osd_order(a, count, (hipStream_t)stream));
  return QLDPC_OK;
}

extern "C" int qldpc_osd_device_ordered(const qldpc_code* code, int64_t count, const uint8_t* d_syn,
                                        const double* d_post, int order, uint8_t* d_ehat, int32_t* d_status,
                                        int32_t* d_perm, int32_t* d_tiepos, void* stream) {
  return qldpc_osd_device_ordered_ex(code, count, d_syn, d_post, order, d_ehat, d_status, d_perm, d_tiepos,
                                     nullptr, nullptr, nullptr, 0, stream);
}

extern "C" int qldpc_osd_device_ordered_ex(const qldpc_code* code, int64_t count, const uint8_t* d_syn,
                                           const double* d_post, int order, uint8_t* d_ehat, int32_t* d_status,
                                           int32_t* d_perm, int32_t* d_tiepos, double* d_spill_post,
                                           int32_t* d_spill_idx, int32_t* d_spill_count, int64_t spill_cap,
                                           void* stream) {
  if (d_spill_count && (!d_spill_post || !d_spill_idx || spill_cap < 0))
    return fail(QLDPC_EINVAL, "spill buffers incomplete");
  if (d_spill_count && count > INT32_MAX) return fail(QLDPC_EINVAL, "spill indices are int32");
  int rc = qldpc_osd_order_device(code, count, d_post, d_perm, d_tiepos, stream);
  if (rc != QLDPC_OK) return rc;
  g_spill = {d_spill_post, d_spill_idx, d_spill_count, spill_cap};
  rc = osd_device_impl(code, count, d_syn, d_perm, d_tiepos, d_post, order, d_ehat, d_status, stream);
  g_spill = {};
  return rc;
}

// osd_hbm_kernel: one workgroup per shot, the shot's working matrix in a
// per-shot slice of a stream-ordered scratch allocation (chunks of at most
// 1 GiB of slices), LDS = one 64-bit word per row + small
static int osd_hbm_impl(const qldpc_code* code, int64_t count, const uint8_t* d_syn, const int32_t* d_perm,
                        const int32_t* d_tiepos, const double* d_post, int order, uint8_t* d_ehat,
                        int32_t* d_status, void* stream) {
  const int m = code->m, n = code->n;
  const int nwr = (n + 1 + 63) / 64, mp = (m + 63) / 64 * 64;
  int dev = 0, max_lds = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  const size_t lds = qldpc::osd_hbm_lds(m, nwr);
  if (lds > (size_t)max_lds)
    return fail(QLDPC_EUNSUP, "GPU OSD keeps one word per row in LDS: m = %d needs %zu B (at most %d)", m, lds,
                max_lds);
  const void* k = qldpc::osd_hbm_kernel_ptr();
  HIP_TRY(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  code_osd_prep(code);
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  qldpc::OsdHbmArgs h{};
  size_t off = up((size_t)8 * nwr * mp);
  h.off_inv = (int)off;
  off = up(off + 4 * (size_t)n);
  h.off_jl = (int)off;
  off = up(off + 4 * ((size_t)m + 2));
  h.off_inj = (int)off;
  off = up(off + (size_t)n);
  h.off_table = (int)off;
  if (order == 1) off = up(off + 4 * (size_t)setdiff_table_ints(n));
  if (off > (size_t)INT32_MAX) return fail(QLDPC_EUNSUP, "GPU OSD scratch per shot exceeds 2 GiB (m = %d, n = %d)", m, n);
  h.stride = (long long)off;
  h.nwr = nwr;
  h.mp = mp;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(count, 1 << 30),
                                                                   ((int64_t)1 << 30) / (int64_t)off));
  void* scr = nullptr;
  HIP_TRY(hipMallocAsync(&scr, (size_t)chunk * off, (hipStream_t)stream));
  h.scratch = (unsigned char*)scr;
  qldpc::OsdArgs a{};
  a.row_ptr = code->d_row_ptr;
  a.col_idx = code->d_col_idx;
  a.m = m;
  a.n = n;
  a.rank = code->rank;
  a.order = order;
  a.post = d_tiepos ? d_post : nullptr;
  if (d_tiepos && g_spill.count) {
    a.spill_post = g_spill.post;
    a.spill_idx = g_spill.idx;
    a.spill_count = g_spill.count;
    a.spill_cap = g_spill.cap;
  }
  const int block = std::min(1024, std::max(64, mp));
  hipError_t e = hipSuccess;
  for (int64_t done = 0; done < count && e == hipSuccess; done += chunk) {
    const int64_t g = std::min<int64_t>(count - done, chunk);
    qldpc::OsdArgs ai = a;
    ai.perm = d_perm + done * n;
    ai.syn = d_syn + done * m;
    ai.ehat = d_ehat + done * n;
    ai.status = d_status + done;
    ai.tiepos = d_tiepos ? d_tiepos + done : nullptr;
    if (ai.post) ai.post = d_post + done * n;
    ai.shot_base = done;
    void* params[] = {(void*)&ai, (void*)&h};
    e = hipLaunchKernel(k, dim3((unsigned)g), dim3(block), params, lds, (hipStream_t)stream);
  }
  const hipError_t ef = hipFreeAsync(scr, (hipStream_t)stream);
  HIP_TRY(e);
  HIP_TRY(ef);
  return QLDPC_OK;
}

static int osd_device_impl(const qldpc_code* code, int64_t count, const uint8_t* d_syn, const int32_t* d_perm,
                           const int32_t* d_tiepos, const double* d_post, int order, uint8_t* d_ehat,
                           int32_t* d_status, void* stream) {
  if (!code) return fail(QLDPC_EINVAL, "code is null");
  if (count < 0) return fail(QLDPC_EINVAL, "negative count");
  if (count == 0) return QLDPC_OK;
  if (code->device < 0) return fail(QLDPC_EHIP, "no HIP device was visible when the code was created");
  if (!d_syn || !d_perm || !d_ehat || !d_status) return fail(QLDPC_EINVAL, "null device buffer");
  const int m = code->m, n = code->n;
  const int nw = qldpc::osd_nw_of((n + 1 + 63) / 64);
  const void* kcol = qldpc::select_osd_kernel(nw);
  // past the register / LDS kernels (m > 1024 rows, n > 2111 columns), or
  // option osd_hbm: the working matrix in global memory (osd_hbm_kernel)
  if (m > 1024 || !kcol || opt(&Options::osd_hbm) != 0)
    return osd_hbm_impl(code, count, d_syn, d_perm, d_tiepos, d_post, order, d_ehat, d_status, stream);
  // The block kernel picks pivot rows by row index instead of REF's row
  // order: same J, same e_J (the unique solution), except when column 0 of
  // H[:, perm] has no pivot (an all-zero column of H: column kernel for the
  // whole code) or the syndrome lies outside H's column space (the block
  // kernel marks those shots, a second column-kernel pass redoes them).
  // option osd_column: the column kernel alone (A/B reference, tests).
  const bool column = opt(&Options::osd_column) != 0 || code->zero_col;
  int rt = 1;                                        // block kernel: rows per thread
  const void* kblk = column ? nullptr : qldpc::select_osd_block_kernel(nw, m, &rt);
  const int block = std::max(64, (m + 63) / 64 * 64);
  const int bblk = std::max(64, ((m + rt - 1) / rt + 63) / 64 * 64);   // block kernel threads
  const int mr = rt * bblk;                          // its row slots
  const int base = align16(4 * n + 4 * (m + 2) + n) + (order == 1 ? 4 * setdiff_table_ints(n) : 0);
  const int lds_col = base + 8 * nw * (1 + 2 * 16 + 2) + 4 * 32 + 16;         // emask, candidate / xrow rows, slots, misc
  const int lds_blk = base + 8 * nw * (1 + 64 + (QLDPC_OSD_PAIRS ? 32 : 0)) + 8 * 64 + 8 * 2 * mr + 4 * 3 * mr + 4 * 64 + 64;
                      // emask, PW, PX, CT, Wd / Cm, pkof / pidx / crow, pk, misc
  int dev = 0, max_lds = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  if (lds_col > max_lds) return fail(QLDPC_EUNSUP, "GPU OSD needs %d B LDS", lds_col);
  HIP_TRY(hipFuncSetAttribute(kcol, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  if (kblk && lds_blk > max_lds) kblk = nullptr;
  if (kblk) HIP_TRY(hipFuncSetAttribute(kblk, hipFuncAttributeMaxDynamicSharedMemorySize, max_lds));
  // rank(H) and the column bit-vectors: built on first use, after every
  // cheap refusal above (a large HBM-path code is refused without them)
  code_osd_prep(code);
  qldpc::OsdArgs a{};
  a.row_ptr = code->d_row_ptr;
  a.col_idx = code->d_col_idx;
  a.perm = d_perm;
  a.syn = d_syn;
  a.ehat = d_ehat;
  a.status = d_status;
  a.m = m;
  a.n = n;
  a.rank = code->rank;
  a.order = order;
  a.tiepos = d_tiepos;
  a.post = d_tiepos ? d_post : nullptr;
  if (d_tiepos && g_spill.count) {
    a.spill_post = g_spill.post;
    a.spill_idx = g_spill.idx;
    a.spill_count = g_spill.count;
    a.spill_cap = g_spill.cap;
  }
  static unsigned long long* d_prof = nullptr;       // diagnostic builds (QLDPC_OSD_TIMING)
  if (opt(&Options::osd_prof) && !d_prof) {
    HIP_TRY(hipMalloc(&d_prof, 16 * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(d_prof, 0, 16 * sizeof(unsigned long long)));
  }
  a.prof = d_prof;
  {
    // per-CU workgroup tickets of osd_block_kernel (engine SIMD choice), one
    // zeroed array per device; the counters only ever wrap
    static std::mutex mu;
    static uint32_t* tickets[64] = {};
    std::lock_guard<std::mutex> lk(mu);
    const bool use_tickets = opt(&Options::osd_tickets) != 0;
    if (dev >= 0 && dev < 64 && !tickets[dev] && use_tickets) {
      HIP_TRY(hipMalloc(&tickets[dev], sizeof(uint32_t) * qldpc::kOsdCuSlots));
      HIP_TRY(hipMemset(tickets[dev], 0, sizeof(uint32_t) * qldpc::kOsdCuSlots));
    }
    a.cu_tickets = (dev >= 0 && dev < 64 && use_tickets) ? tickets[dev] : nullptr;
  }
  int64_t done = 0;
  while (done < count) {  // grid.x limit
    const int64_t g = std::min<int64_t>(count - done, 1 << 30);
    qldpc::OsdArgs ai = a;
    ai.perm = d_perm + done * n;
    ai.syn = d_syn + done * m;
    ai.ehat = d_ehat + done * n;
    ai.status = d_status + done;
    if (ai.tiepos) ai.tiepos = d_tiepos + done;
    if (ai.post) ai.post = d_post + done * n;
    ai.shot_base = done;
    void* params[] = {(void*)&ai};
    if (kblk) {
      HIP_TRY(hipLaunchKernel(kblk, dim3((unsigned)g), dim3(bblk), params, (size_t)lds_blk, (hipStream_t)stream));
      ai.redo = 1;                                    // same stream: runs after the block pass
    }
    HIP_TRY(hipLaunchKernel(kcol, dim3((unsigned)g), dim3(block), params, (size_t)lds_col, (hipStream_t)stream));
    done += g;
  }
  if (d_prof) {
    unsigned long long h[16];
    HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
    HIP_TRY(hipMemcpy(h, d_prof, sizeof(h), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(d_prof, 0, sizeof(h)));
    fprintf(stderr, "osd_prof shots=%lld", (long long)count);
    for (int i = 0; i < 14; ++i) fprintf(stderr, " %.0f", (double)h[i] / (double)count);
    fprintf(stderr, "\n");
  }
  return QLDPC_OK;
}

// ---------------------------------------------------------------------------
// device channel sampler and outcome counters (channel_kernels.hip)
// ---------------------------------------------------------------------------
static int pair_tabs(const qldpc_code* hx, const qldpc_code* hz, qldpc::PairTabs* t) {
  if (!hx || !hz) return fail(QLDPC_EINVAL, "code is null");
  if (hx->n != hz->n)
    return fail(QLDPC_EINVAL, "Hx and Hz must have the same number of columns (physical qubits).");
  if (hx->device < 0 || hz->device < 0)
    return fail(QLDPC_EHIP, "no HIP device was visible when the code was created");
  if (hx->device != hz->device) return fail(QLDPC_EINVAL, "Hx and Hz live on different devices");
  const int W = (hx->n + 63) / 64;
  if (W > 64) return fail(QLDPC_EUNSUP, "the channel kernels support n <= 4096 qubits (got %d)", hx->n);
  t->rp_x = hx->d_row_ptr;
  t->ci_x = hx->d_col_idx;
  t->rp_z = hz->d_row_ptr;
  t->ci_z = hz->d_col_idx;
  t->mx = hx->m;
  t->mz = hz->m;
  t->ex = hx->E;
  t->ez = hz->E;
  t->n = hx->n;
  t->W = W;
  t->udeg = (hx->uniform_deg == hz->uniform_deg && hx->m > 0 && hz->m > 0) ? hx->uniform_deg : 0;
  int dev = 0, max_lds = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  if (qldpc::channel_lds_bytes(*t, true) > max_lds)
    return fail(QLDPC_EUNSUP, "the channel kernels need %d B of LDS for these codes",
                qldpc::channel_lds_bytes(*t, true));
  return QLDPC_OK;
}

static int channel_grid(int64_t batch) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  const int64_t need = (batch + qldpc::kChannelWaves - 1) / qldpc::kChannelWaves;
  return (int)std::max<int64_t>(1, std::min<int64_t>(need, (int64_t)cus * 8));
}

extern "C" int qldpc_channel_thresholds(double p, uint64_t* t1, uint64_t* t2, uint64_t* t3) {
  if (!(p >= 0.0 && p <= 1.0)) return fail(QLDPC_EINVAL, "p must lie in [0, 1] (got %g)", p);
  const double q = p / 3.0, two32 = 4294967296.0;
  uint64_t t[3];
  for (int k = 0; k < 3; ++k) t[k] = (uint64_t)std::min(two32, std::floor((k + 1) * q * two32));
  if (t1) *t1 = t[0];
  if (t2) *t2 = t[1];
  if (t3) *t3 = t[2];
  return QLDPC_OK;
}

extern "C" int qldpc_channel_sample(const qldpc_code* hx, const qldpc_code* hz, double p, uint64_t seed,
                                    uint64_t shot0, int64_t batch, uint64_t* d_errx, uint64_t* d_errz,
                                    uint8_t* d_syn_z, uint8_t* d_syn_x, void* stream) {
  return qldpc_channel_sample_ex(hx, hz, p, seed, shot0, batch, d_errx, d_errz, d_syn_z, d_syn_x,
                                 QLDPC_FMT_BYTES, stream);
}

extern "C" int qldpc_channel_sample_ex(const qldpc_code* hx, const qldpc_code* hz, double p, uint64_t seed,
                                       uint64_t shot0, int64_t batch, uint64_t* d_errx, uint64_t* d_errz,
                                       void* d_syn_z, void* d_syn_x, int syn_format, void* stream) {
  if (syn_format != QLDPC_FMT_BYTES && syn_format != QLDPC_FMT_BITS) return fail(QLDPC_EINVAL, "unknown syndrome format");
  qldpc::SampleArgs a{};
  int rc = pair_tabs(hx, hz, &a.t);
  if (rc != QLDPC_OK) return rc;
  if (batch < 0) return fail(QLDPC_EINVAL, "negative batch");
  rc = qldpc_channel_thresholds(p, &a.t1, &a.t2, &a.t3);
  if (rc != QLDPC_OK) return rc;
  if (batch == 0) return QLDPC_OK;
  if (!d_errx || !d_errz || (a.t.mz && !d_syn_z) || (a.t.mx && !d_syn_x))
    return fail(QLDPC_EINVAL, "null device buffer");
  a.errx = d_errx;
  a.errz = d_errz;
  a.syz = (uint8_t*)d_syn_z;
  a.syx = (uint8_t*)d_syn_x;
  a.syn_bits = syn_format == QLDPC_FMT_BITS;
  a.batch = batch;
  a.shot0 = shot0;
  a.key0 = (uint32_t)seed;
  a.key1 = (uint32_t)(seed >> 32);
  HIP_TRY(qldpc::launch_channel_sample(a, channel_grid(batch), (hipStream_t)stream));
  return QLDPC_OK;
}

extern "C" int qldpc_count_outcomes(const qldpc_code* hx, const qldpc_code* hz, int64_t batch,
                                    const uint64_t* d_errx, const uint64_t* d_errz, const uint8_t* d_syn_z,
                                    const uint8_t* d_syn_x, const uint8_t* d_ehat_x, const uint8_t* d_ehat_z,
                                    const int32_t* d_iters_x, const int32_t* d_iters_z, int64_t* d_counters,
                                    void* stream) {
  return qldpc_count_outcomes_ex(hx, hz, batch, d_errx, d_errz, d_syn_z, d_syn_x, QLDPC_FMT_BYTES, d_ehat_x,
                                 d_ehat_z, QLDPC_FMT_BYTES, d_iters_x, d_iters_z, d_counters, stream);
}

extern "C" int qldpc_count_outcomes_ex(const qldpc_code* hx, const qldpc_code* hz, int64_t batch,
                                       const uint64_t* d_errx, const uint64_t* d_errz, const void* d_syn_z,
                                       const void* d_syn_x, int syn_format, const void* d_ehat_x,
                                       const void* d_ehat_z, int ehat_format, const int32_t* d_iters_x,
                                       const int32_t* d_iters_z, int64_t* d_counters, void* stream) {
  if ((syn_format != QLDPC_FMT_BYTES && syn_format != QLDPC_FMT_BITS) ||
      (ehat_format != QLDPC_FMT_BYTES && ehat_format != QLDPC_FMT_BITS))
    return fail(QLDPC_EINVAL, "unknown syndrome / estimate format");
  qldpc::CountArgs a{};
  int rc = pair_tabs(hx, hz, &a.t);
  if (rc != QLDPC_OK) return rc;
  if (batch < 0) return fail(QLDPC_EINVAL, "negative batch");
  if (batch == 0) return QLDPC_OK;
  if (!d_errx || !d_errz || (a.t.mz && !d_syn_z) || (a.t.mx && !d_syn_x) || !d_ehat_x || !d_ehat_z ||
      !d_iters_x || !d_iters_z || !d_counters)
    return fail(QLDPC_EINVAL, "null device buffer");
  a.errx = d_errx;
  a.errz = d_errz;
  a.syz = (const uint8_t*)d_syn_z;
  a.syx = (const uint8_t*)d_syn_x;
  a.ehx = (const uint8_t*)d_ehat_x;
  a.ehz = (const uint8_t*)d_ehat_z;
  a.syn_bits = syn_format == QLDPC_FMT_BITS;
  a.eh_bits = ehat_format == QLDPC_FMT_BITS;
  a.itx = d_iters_x;
  a.itz = d_iters_z;
  a.acc = reinterpret_cast<unsigned long long*>(d_counters);
  a.batch = batch;
  HIP_TRY(qldpc::launch_count_outcomes(a, channel_grid(batch), (hipStream_t)stream));
  return QLDPC_OK;
}
