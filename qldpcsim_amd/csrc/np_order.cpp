// np_order.cpp — the OSD reliability order exactly as NumPy computes it on the
// reference's host (decoders.py:320-325):
//     perm = np.argsort(np.where(prob > 0.5, prob, 1 - prob)),
//     prob = 1 / (1 + np.exp(clip(P, -100, 100)))
// The keys come from include/qldpc_libm.h (qldpc_osd_key: SVML exp8_ha
// restated). np.argsort's default kind on NumPy 2.2.6 / x86-64 AVX512_SKX is
// x86-simd-sort's 64-bit argsort (np::qsort_simd::ArgQSort_AVX512_SKX<double>,
// vendored in NumPy, BSD-3), whose handling of equal keys IS the order of tied
// reliabilities; it is restated here step for step (read from the dispatched
// machine code, pinned by tests/test_osd_order.py against np.argsort itself):
//
//   ArgQSort(arr, arg, n): n <= 1 -> done; any NaN -> std::sort with a NaN
//     comparator (not restated: status 1); else
//     argsort_64bit_(arr, arg, 0, n - 1, max_iters = 2 * floor(log2 n)).
//   argsort_64bit_(L, R, it):
//     it <= 0           -> std::sort of the range (not restated: status 1)
//     R + 1 - L <= 256  -> argsort_n: bitonic network on P = max(8, 2^ceil)
//                          slots, +inf padding, "flip + half-cleaner" stages,
//                          every comparator (lo, hi) moving the pair only if
//                          key[hi] < key[lo] (ties never move)
//     else pivot = 5th smallest of the keys at L + q, L + 2q .. L + 8q
//          (q = (R - L) / 8); argpartition_unrolled<4> (below) -> pidx;
//          pivot != min -> recurse (L, pidx - 1, it - 1);
//          pivot != max -> recurse (pidx, R, it - 1)
//   argpartition_unrolled<4> on [left, right):
//     (right - left) % 32 scalar steps from the left: key >= pivot ->
//       swap(arg[left], arg[--right]), else ++left;
//     then 32-element blocks: the first and last block are held back; the
//     middle blocks are consumed from the left or from the right (right when
//     fewer elements have been stored on the right than on the left), each as
//     four 8-lane vectors, then the held-back first and last blocks; a vector
//     compress-stores its < pivot lanes (lane order) at l_store and its
//     >= pivot lanes (lane order) just below r_store + 8, then l_store +=
//     #lt, r_store -= #ge; returns l_store.
// The device kernel (osd_kernels.hip, osd_order_kernel) runs the same
// algorithm with a workgroup per shot.

#include <hip/hip_runtime.h>
#include <math.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/qldpc_decoder.h"
#include "../../include/qldpc_libm.h"

namespace {

struct NpOrder {
  const double* key;
  int32_t* arg;
  std::vector<int32_t> snap;
  bool fallback = false;

  void cmpx(int lo, int hi) {
    const int32_t a = arg[lo], b = arg[hi];
    if (key[b] < key[a]) {
      arg[lo] = b;
      arg[hi] = a;
    }
  }

  // argsort_n_vec: bitonic network over P slots, virtual +inf pads (a pad never
  // moves and never displaces a real key: comparators with hi >= N are no-ops)
  void small(int L, int N) {
    int P = 8;
    while (P < N) P <<= 1;
    for (int k = 2; k <= P; k <<= 1) {
      for (int x = 0; x < P; ++x) {
        const int y = x ^ (k - 1);
        if (x < y && y < N) cmpx(L + x, L + y);
      }
      for (int j = k >> 2; j >= 1; j >>= 1)
        for (int x = 0; x < P; ++x) {
          const int y = x ^ j;
          if (x < y && y < N) cmpx(L + x, L + y);
        }
    }
  }

  void sort(int L, int R, int it) {
    if (it <= 0) {
      fallback = true;          // std_argsort (libstdc++ introsort): not restated
      return;
    }
    if (R + 1 - L <= 256) {
      small(L, R + 1 - L);
      return;
    }
    const int d = R - L, q = d >> 3;
    double s[8];
    for (int i = 0; i < 8; ++i) s[i] = key[arg[L + q * (i + 1)]];
    std::sort(s, s + 8);
    const double pivot = s[4];
    double smallest = INFINITY, biggest = -INFINITY;
    int left = L, right = R + 1;
    for (int i = (right - left) % 32; i > 0; --i) {
      const double v = key[arg[left]];
      smallest = std::min(v, smallest);
      biggest = std::max(v, biggest);
      if (!(v < pivot)) std::swap(arg[left], arg[--right]);
      else ++left;
    }
    snap.assign(arg + left, arg + right);
    const int base = left;
    int l_store = left, r_store = right - 8;
    auto vec = [&](int pos) {
      int ge[8], lt[8], ng = 0, nl = 0;
      for (int i = 0; i < 8; ++i) {
        const int32_t a = snap[pos - base + i];
        const double v = key[a];
        smallest = std::min(v, smallest);
        biggest = std::max(v, biggest);
        if (v >= pivot) ge[ng++] = a;
        else lt[nl++] = a;
      }
      for (int i = 0; i < nl; ++i) arg[l_store + i] = lt[i];
      for (int i = 0; i < ng; ++i) arg[r_store + 8 - ng + i] = ge[i];
      l_store += nl;
      r_store -= ng;
    };
    const int first = left, last = right - 32;
    left += 32;
    right -= 32;
    while (right != left) {
      int blk;
      if ((r_store + 8) - right < left - l_store) {
        right -= 32;
        blk = right;
      } else {
        blk = left;
        left += 32;
      }
      for (int v = 0; v < 4; ++v) vec(blk + 8 * v);
    }
    for (int v = 0; v < 4; ++v) vec(first + 8 * v);
    for (int v = 0; v < 4; ++v) vec(last + 8 * v);
    const int pidx = l_store;
    if (pivot != smallest) sort(L, pidx - 1, it - 1);
    if (pivot != biggest) sort(pidx, R, it - 1);
  }
};

}  // namespace

// Host threads this process may use (qldpcsim_amd/hostcores.py's
// process_cores): the affinity mask, capped by the cgroup CPU quota
// (cpu.max) and by OMP_NUM_THREADS — not hardware_concurrency(), which counts
// CPUs the process may not run on.
int qldpc_host_thread_budget() {
  int n = (int)std::max(1u, std::thread::hardware_concurrency());
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[64] = {0};
    double per = 0;
    if (fscanf(f, "%63s %lf", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
      n = std::min(n, std::max(1, (int)(atof(q) / per)));
    fclose(f);
  }
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const int o = atoi(e);
    if (o > 0) n = std::min(n, o);
  }
  return n;
}


// One row: keys from the posteriors, NumPy's argsort. 0 = exact, 1 = a case
// this restatement leaves to NumPy (a NaN key, or x86-simd-sort's std::sort
// fallback after 2 floor(log2 n) levels).
static int np_order_row(const double* post, int n, int32_t* perm, double* key) {
  bool nan = false;
  for (int i = 0; i < n; ++i) {
    key[i] = qldpc_osd_key(post[i]);
    nan |= key[i] != key[i];
    perm[i] = i;
  }
  if (n <= 1) return 0;
  if (nan) return 1;
  NpOrder o{key, perm, {}};
  int lg = 0;
  while ((2 << lg) <= n) ++lg;                         // floor(log2 n)
  o.sort(0, n - 1, 2 * lg);
  return o.fallback ? 1 : 0;
}

extern "C" int qldpc_osd_order_host(const double* h_post, int64_t count, int n, int32_t* h_perm,
                                    int32_t* h_status, int nthreads) {
  if (count < 0 || n < 0) return QLDPC_EINVAL;
  if (count == 0 || n == 0) return QLDPC_OK;
  if (!h_post || !h_perm || !h_status) return QLDPC_EINVAL;
  if (nthreads <= 0) nthreads = qldpc_host_thread_budget();
  nthreads = (int)std::min<int64_t>(nthreads, count);
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    std::vector<double> key((size_t)n);
    while (true) {
      const int64_t b = next.fetch_add(1);
      if (b >= count) return;
      h_status[b] = np_order_row(h_post + b * (int64_t)n, n, h_perm + b * (int64_t)n, key.data());
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  return QLDPC_OK;
}

extern "C" int qldpc_np_argsort_host(const double* h_key, int n, int32_t* h_perm) {
  if (n < 0 || (n && (!h_key || !h_perm))) return QLDPC_EINVAL;
  for (int i = 0; i < n; ++i) {
    if (h_key[i] != h_key[i]) return 1;
    h_perm[i] = i;
  }
  if (n <= 1) return 0;
  NpOrder o{h_key, h_perm, {}};
  int lg = 0;
  while ((2 << lg) <= n) ++lg;
  o.sort(0, n - 1, 2 * lg);
  return o.fallback ? 1 : 0;
}

extern "C" void qldpc_osd_keys_host(const double* h_post, int64_t count, double* h_key, int exp_only) {
  if (exp_only)
    for (int64_t i = 0; i < count; ++i) h_key[i] = qldpc_np_exp(h_post[i]);
  else
    for (int64_t i = 0; i < count; ++i) h_key[i] = qldpc_osd_key(h_post[i]);
}

// The restated NumPy libm BP and the priors run (include/qldpc_libm.h, the
// same code the kernels compile), element-wise on the host: the run-time pin
// decoders.numpy_libm_pinned() compares it with the running NumPy.
extern "C" int qldpc_libm_eval_host(int fn, const double* h_x, int64_t count, double* h_y) {
  if (count < 0 || (count && (!h_x || !h_y))) return QLDPC_EINVAL;
  switch (fn) {
    case QLDPC_LIBM_TANH:  for (int64_t i = 0; i < count; ++i) h_y[i] = qldpc_tanh(h_x[i]); break;
    case QLDPC_LIBM_ATANH: for (int64_t i = 0; i < count; ++i) h_y[i] = qldpc_atanh(h_x[i]); break;
    case QLDPC_LIBM_LOG:   for (int64_t i = 0; i < count; ++i) h_y[i] = qldpc_np_log(h_x[i]); break;
    case QLDPC_LIBM_EXP:   for (int64_t i = 0; i < count; ++i) h_y[i] = qldpc_np_exp(h_x[i]); break;
    default: return QLDPC_EINVAL;
  }
  return QLDPC_OK;
}
