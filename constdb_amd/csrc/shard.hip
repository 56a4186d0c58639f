// Several GPUs in one process: cdb_ctx_create_multi / cdb_merge_sharded.
//
// The reference merges every snapshot on the single main task of one server process
// (server.rs:95,128-130; replica/pull.rs:120-128). Here one process drives a node's GPUs: a
// multi-device context holds one engine context per device slot and RCCL communicators between
// them (ncclCommInitAll). Keys shard by owner = the top log2(N) bits of the key hash; children
// carry their parent's hash, so a key and its children always meet on one device and every rule
// of SURVEY §8a stays device-local. One step:
//   1. splits  : per device, the owner boundaries of every run (a run is in key-hash order, so the
//                rows a device owes owner d are ONE contiguous slice of each run): one thread per
//                (family, run, owner) binary-searches the run's hash column; the same launch checks
//                that every run is non-decreasing. Inputs not in runs (or found out of order) are
//                grouped by owner first (cdb_partition_owner) and travel as one unsorted "run";
//   2. plan    : on the host (one process sees every split: no count all-to-all), the receive
//                layout of each device -- one run per (source device, source run) that has rows;
//   3. exchange: one RCCL group of point-to-point transfers (per source run, family and column a
//                contiguous slice, in pieces of at most 1 GiB), a device's own slices by device
//                copies. Device slots that share a GPU move rows by device copies instead;
//   4. merge   : every device merges what it received on its own host thread (the pipeline
//                synchronises its stream once midway), with key_shift = log2(N): on the sorted-run
//                path when every source was in runs. Outputs stay on their devices.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "engine.h"

namespace cdb {

// RCCL, loaded on first use: a process that never builds a multi-device context never maps it,
// and one that already holds torch's RCCL (same soname) shares that copy.
struct Node {
  void* lib = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::vector<ncclComm_t> comms;
  bool rccl = false;  // distinct devices: rows move by RCCL; otherwise by device copies
};

void node_destroy(Node* n) {
  if (!n) return;
  if (n->destroy)
    for (ncclComm_t c : n->comms)
      if (c) n->destroy(c);
  delete n;  // (the library stays mapped: RCCL keeps process-wide state)
}

namespace {

#define CDB_SHARD_TRY(...)            \
  do {                                \
    cdb_status _s = (__VA_ARGS__);    \
    if (_s != CDB_OK) return _s;      \
  } while (0)
#define CDB_SHARD_HIP(c, x, what) CDB_SHARD_TRY(fail_from((c), hip_check((c), (x), (what))))
#define CDB_SHARD_NCCL(x, what) CDB_SHARD_TRY(nccl_check(ctx, node, (x), (what)))

constexpr uint64_t kMaxPieceRows = (1ull << 30) / 8;  // 1 GiB per transfer

cdb_ctx* slot_ctx(cdb_ctx* ctx, int i) { return i == 0 ? ctx : ctx->shards[i - 1]; }

int slot_count(const cdb_ctx* ctx) { return 1 + (int)ctx->shards.size(); }

// RCCL's library: CDB_RCCL_LIB names it (tests point it at a missing file), else the soname, else
// ROCm's copy. Returns an empty string, or what failed.
std::string load_rccl(Node* n) {
  const char* path = std::getenv("CDB_RCCL_LIB");
  if (path && path[0]) {
    n->lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  } else {
    n->lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!n->lib) n->lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  }
  if (!n->lib) {
    const char* e = dlerror();
    return std::string("cannot load RCCL: ") + (e ? e : "dlopen failed");
  }
  auto sym = [&](const char* name) { return dlsym(n->lib, name); };
  n->init_all = (decltype(n->init_all))sym("ncclCommInitAll");
  n->destroy = (decltype(n->destroy))sym("ncclCommDestroy");
  n->send = (decltype(n->send))sym("ncclSend");
  n->recv = (decltype(n->recv))sym("ncclRecv");
  n->group_start = (decltype(n->group_start))sym("ncclGroupStart");
  n->group_end = (decltype(n->group_end))sym("ncclGroupEnd");
  n->error_string = (decltype(n->error_string))sym("ncclGetErrorString");
  if (!n->init_all || !n->destroy || !n->send || !n->recv || !n->group_start || !n->group_end)
    return "RCCL lacks the point-to-point API";
  return std::string();
}

cdb_status nccl_check(cdb_ctx* ctx, const Node* n, ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return CDB_OK;
  return fail(ctx, CDB_DEVICE_ERROR,
              std::string(what) + ": " + (n->error_string ? n->error_string(r) : std::to_string((int)r)));
}

// ---- kernels
struct SplitArgs {
  const uint64_t* kh[3];   // column 0 of each family (key hash / parent key hash)
  const uint64_t* rs;      // run starts, [3][R + 1]
  uint32_t R;
  uint32_t world;
  int bits;                // log2(world)
  uint64_t* out;           // [3][R][world + 1] absolute rows: owner d of run r = [out[d], out[d + 1])
  unsigned long long* bad; // set when a run decreases somewhere
  uint64_t n[3];
};

// One thread per (family, run, owner boundary): the run's first row whose owner is >= d.
__global__ void owner_split_kernel(SplitArgs a) {
  const uint32_t per_f = a.R * (a.world + 1);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * per_f) return;
  const uint32_t f = i / per_f, rem = i - f * per_f, r = rem / (a.world + 1), d = rem - r * (a.world + 1);
  const uint64_t lo = a.rs[f * (a.R + 1) + r], hi = a.rs[f * (a.R + 1) + r + 1];
  a.out[i] = d == 0 ? lo : d == a.world ? hi : owner_lower_bound(a.kh[f], lo, hi, d, a.bits);
}

// Every run must be non-decreasing in the key hash. A decreasing adjacent pair is a violation
// unless its second row starts a run (R - 1 such pairs per family in a valid input).
__global__ void __launch_bounds__(256) run_order_kernel(SplitArgs a) {
  const uint64_t total = a.n[0] + a.n[1] + a.n[2];
  bool bad = false;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total; g += (uint64_t)gridDim.x * blockDim.x) {
    const int f = g < a.n[0] ? 0 : g < a.n[0] + a.n[1] ? 1 : 2;
    const uint64_t i = g - (f > 0 ? a.n[0] : 0) - (f > 1 ? a.n[1] : 0);
    if (i + 1 >= a.n[f] || a.kh[f][i] <= a.kh[f][i + 1]) continue;
    bool boundary = false;
    for (uint32_t r = 1; r < a.R; ++r) boundary |= a.rs[f * (a.R + 1) + r] == i + 1;
    bad |= !boundary;
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(a.bad, 1ull);
}

// ---- host side
// One source device's rows as the exchange sees them: R runs per family (or one owner-grouped
// "run" when the input was not in sorted runs), with the owner splits of every run.
struct Source {
  uint32_t R = 0;
  bool sorted = false;
  std::vector<uint64_t> rs;   // [3][R + 1] run starts (device-upload copy)
  std::vector<uint64_t> sp;   // [3][R][N + 1] absolute rows of each owner slice
  unsigned long long bad = 0;
  const uint64_t* cols[3][8] = {};
  uint32_t stride[3] = {1, 1, 1};  // record stride per family (1: columns)
  uint64_t split(int f, uint32_t r, int d, int N) const { return sp[((uint64_t)f * R + r) * (N + 1) + d]; }
};

constexpr int kFamCols[3] = {kKeyCols, kNodeCols, kMemberCols};
constexpr int kOutCols[3] = {kKeyOutCols, kNodeCols, kMemberCols};

const cdb_dev_rows& fam_rows(const cdb_dev_input& d, int f) { return f == 0 ? d.keys : f == 1 ? d.nodes : d.members; }

bool runs_valid(const cdb_dev_input& d) {
  if (d.n_runs < 1 || d.n_runs > CDB_MAX_RUNS) return false;
  for (int f = 0; f < 3; ++f) {
    const uint64_t* rs = d.run_start[f];
    if (rs[0] != 0 || rs[d.n_runs] != fam_rows(d, f).n) return false;
    for (uint32_t r = 0; r < d.n_runs; ++r)
      if (rs[r] > rs[r + 1]) return false;
  }
  return true;
}

// Columns of `rows` rows x ncols u64 in workspace slot `slot` of c.
cdb_status ws_cols(cdb_ctx* c, int slot, int ncols, uint64_t rows, uint64_t** col) {
  cdb_status st = CDB_OK;
  const uint64_t n = std::max<uint64_t>(rows, 1);
  uint64_t* p = (uint64_t*)ws_get(c, slot, ncols * n * sizeof(uint64_t), &st);
  if (!p) return st;
  for (int k = 0; k < ncols; ++k) col[k] = p + k * n;
  return CDB_OK;
}

// Rows of one family in workspace slot `slot` of c, in the given layout (stride 1: columns; else
// the records layout: a hash column, then records of `stride` words starting 16-B aligned).
cdb_status ws_rows(cdb_ctx* c, int slot, int ncols, uint64_t rows, uint32_t stride, cdb_dev_rows* r) {
  std::memset(r, 0, sizeof *r);
  if (stride <= 1) return ws_cols(c, slot, ncols, rows, r->col);
  cdb_status st = CDB_OK;
  const uint64_t n = std::max<uint64_t>(rows, 1), hw = (n + 1) & ~1ull;
  uint64_t* p = (uint64_t*)ws_get(c, slot, (hw + (uint64_t)stride * n + 2) * sizeof(uint64_t), &st);
  if (!p) return st;
  r->col[0] = p;
  for (int k = 1; k < ncols; ++k) r->col[k] = p + hw + (k - 1);
  r->stride = stride;
  return CDB_OK;
}

// Arrays a family's rows move as: columns, one per field; records, the hash column and the
// records (so a slice of rows [a, e) is one contiguous range of each array).
int fam_arrays(int f, uint32_t stride) { return stride > 1 ? 2 : kFamCols[f]; }
uint64_t array_words(int k, uint32_t stride) { return (k > 0 && stride > 1) ? stride : 1; }

}  // namespace
}  // namespace cdb

extern "C" cdb_status cdb_shard_recv_plan(uint32_t n_sources, const uint32_t* n_runs, const uint64_t* counts,
                                          uint32_t cap, uint32_t* n_recv_runs, uint32_t* recv_src,
                                          uint32_t* recv_run, uint64_t* run_start, uint64_t* totals) {
  if (!n_runs || !counts || !n_recv_runs || !totals || (cap && (!recv_src || !recv_run || !run_start)))
    return CDB_BAD_ARGUMENT;
  uint32_t k = 0;
  uint64_t acc[3] = {0, 0, 0};
  const uint64_t* c = counts;  // source i's [3][R_i]
  for (uint32_t i = 0; i < n_sources; ++i) {
    const uint32_t R = n_runs[i];
    for (uint32_t r = 0; r < R; ++r) {
      const uint64_t n0 = c[r], n1 = c[R + r], n2 = c[2 * R + r];
      if (!(n0 | n1 | n2)) continue;
      if (k < cap) {
        recv_src[k] = i;
        recv_run[k] = r;
        run_start[k] = acc[0];
        run_start[(cap + 1) + k] = acc[1];
        run_start[2 * (cap + 1) + k] = acc[2];
      }
      acc[0] += n0;
      acc[1] += n1;
      acc[2] += n2;
      ++k;
    }
    c += 3ull * R;
  }
  if (k <= cap)
    for (int f = 0; f < 3; ++f) run_start[f * (uint64_t)(cap + 1) + k] = acc[f];
  *n_recv_runs = k;
  for (int f = 0; f < 3; ++f) totals[f] = acc[f];
  return k <= cap ? CDB_OK : CDB_BAD_ARGUMENT;
}

extern "C" cdb_status cdb_shard_splits(const uint64_t* kh, const uint64_t* run_start, uint32_t n_runs,
                                       uint32_t n_devices, uint64_t* out) {
  if (!run_start || !out || n_devices < 1 || n_devices > 256 || (n_devices & (n_devices - 1))) return CDB_BAD_ARGUMENT;
  int bits = 0;
  while ((1u << bits) < n_devices) ++bits;
  for (uint32_t r = 0; r < n_runs; ++r) {
    const uint64_t lo = run_start[r], hi = run_start[r + 1];
    if (hi < lo || (hi > lo && !kh)) return CDB_BAD_ARGUMENT;
    for (uint32_t d = 0; d <= n_devices; ++d)
      out[(uint64_t)r * (n_devices + 1) + d] = d == 0 ? lo : d == n_devices ? hi : cdb::owner_lower_bound(kh, lo, hi, d, bits);
  }
  return CDB_OK;
}

namespace cdb {
namespace {

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace
}  // namespace cdb

using namespace cdb;

extern "C" {

cdb_status cdb_ctx_create_multi(cdb_ctx** out, int device_count, const int* devices) {
  if (!out) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if (!devices || device_count < 1 || device_count > 8 || (device_count & (device_count - 1))) return CDB_BAD_ARGUMENT;
  bool distinct = true;
  for (int i = 0; i < device_count; ++i)
    for (int j = 0; j < i; ++j) distinct = distinct && devices[i] != devices[j];
  // Distinct GPUs exchange rows over RCCL point-to-point. A context whose RCCL cannot be loaded or
  // whose communicators cannot be created is refused (CDB_DEVICE_ERROR, the reason in
  // cdb_last_error(NULL)): a node would otherwise merge over another transport than the one asked
  // for. CDB_SHARD_TRANSPORT=peer selects HIP peer copies over the same links explicitly
  // (transport 2 in cdb_exchange_stats). RCCL is loaded before any device is touched.
  const char* tr = std::getenv("CDB_SHARD_TRANSPORT");
  const bool want_rccl = device_count > 1 && distinct && !(tr && std::strcmp(tr, "peer") == 0);
  Node* node = new Node();
  if (want_rccl) {
    const std::string why = load_rccl(node);
    if (!why.empty()) {
      node_destroy(node);
      return set_create_error(CDB_DEVICE_ERROR, why + " (CDB_SHARD_TRANSPORT=peer selects HIP peer copies)");
    }
  }
  cdb_ctx* root = nullptr;
  cdb_status st = cdb_ctx_create(&root, devices[0]);
  if (st != CDB_OK) {
    node_destroy(node);
    return set_create_error(st, "device " + std::to_string(devices[0]) + " unavailable");
  }
  root->node = node;
  for (int i = 1; i < device_count; ++i) {
    cdb_ctx* c = nullptr;
    if ((st = cdb_ctx_create(&c, devices[i])) != CDB_OK) {
      cdb_ctx_destroy(root);
      return set_create_error(st, "device " + std::to_string(devices[i]) + " unavailable");
    }
    root->shards.push_back(c);
  }
  if (want_rccl) {
    node->comms.assign(device_count, nullptr);
    if (nccl_check(root, node, node->init_all(node->comms.data(), device_count, devices), "ncclCommInitAll") !=
        CDB_OK) {
      const std::string why = cdb_last_error(root);
      cdb_ctx_destroy(root);
      return set_create_error(CDB_DEVICE_ERROR, why + " (CDB_SHARD_TRANSPORT=peer selects HIP peer copies)");
    }
    node->rccl = true;
  } else if (device_count > 1 && distinct) {
    for (int i = 0; i < device_count; ++i) {  // peer copies, asked for: direct peer access where the links allow it
      hipSetDevice(devices[i]);
      for (int j = 0; j < device_count; ++j) {
        int ok = 0;
        if (i != j && hipDeviceCanAccessPeer(&ok, devices[i], devices[j]) == hipSuccess && ok)
          (void)hipDeviceEnablePeerAccess(devices[j], 0);
      }
    }
    (void)hipGetLastError();
    hipSetDevice(devices[0]);
  }
  *out = root;
  return CDB_OK;
}

int cdb_ctx_device_count(const cdb_ctx* ctx) { return ctx ? slot_count(ctx) : 0; }

cdb_ctx* cdb_ctx_shard(cdb_ctx* ctx, int i) {
  if (!ctx || i < 0 || i >= slot_count(ctx)) return nullptr;
  return slot_ctx(ctx, i);
}

cdb_status cdb_merge_sharded(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts, cdb_dev_output* out,
                             cdb_merge_stats* stats, cdb_exchange_stats* xs) {
  if (!ctx || !in || !out) return CDB_BAD_ARGUMENT;
  const auto t0 = std::chrono::steady_clock::now();
  const int N = slot_count(ctx);
  int bits = 0;
  while ((1 << bits) < N) ++bits;
  const Node* node = ctx->node;
  const bool rccl = node && node->rccl;
  cdb_exchange_stats X;
  std::memset(&X, 0, sizeof X);
  X.n_devices = (uint32_t)N;
  X.transport = N == 1 ? 0 : rccl ? 1 : 2;
  cdb_merge_opts o{};
  if (opts) o = *opts;
  o.key_shift = (uint32_t)bits;
  uint32_t n_pos = 0;
  for (int i = 0; i < N; ++i) n_pos = std::max(n_pos, in[i].n_pos);
  cdb_status st = CDB_OK;
  auto fail_from = [&](cdb_ctx* c, cdb_status e) {
    if (e != CDB_OK && c != ctx) ctx->last_error = "device slot " + std::to_string(c->device) + ": " + c->last_error;
    return e;
  };

  // output columns of slot d for (at most) rows[f] rows
  auto outputs = [&](int d, const uint64_t* rows) -> cdb_status {
    cdb_ctx* c = slot_ctx(ctx, d);
    std::memset(&out[d], 0, sizeof out[d]);
    cdb_dev_rows* o3[3] = {&out[d].keys, &out[d].nodes, &out[d].members};
    const int slots[3] = {WS_YK, WS_YN, WS_YM};
    for (int f = 0; f < 3; ++f)
      if ((st = ws_cols(c, slots[f], kOutCols[f], rows[f], o3[f]->col)) != CDB_OK) return fail_from(c, st);
    out[d].compact = 1;
    return CDB_OK;
  };

  // Inputs must not live in this call's own workspace (a previous call's outputs or received rows):
  // growing a slot would free them under the exchange. Chain through cdb_dev_state_rows instead.
  for (int i = 0; i < N; ++i)
    for (int f = 0; f < 3; ++f) {
      const cdb_dev_rows& r = fam_rows(in[i], f);
      for (int k = 0; k < kFamCols[f] && r.n; ++k)
        for (int j = 0; j < N; ++j)
          for (int slot = WS_XK; slot <= WS_PM; ++slot) {
            const cdb_ctx::Buf& b = slot_ctx(ctx, j)->ws[slot];
            const uintptr_t p = (uintptr_t)r.col[k], lo = (uintptr_t)b.p;
            if (b.p && p >= lo && p < lo + b.bytes)
              return fail(ctx, CDB_BAD_ARGUMENT,
                          "cdb_merge_sharded: an input lies in the library's exchange/output workspace (a previous "
                          "call's output); copy it with cdb_dev_state_rows first");
          }
    }

  if (N == 1) {  // one device: the rows are merged where they lie
    hipSetDevice(ctx->device);
    const uint64_t rows[3] = {in[0].keys.n, in[0].nodes.n, in[0].members.n};
    CDB_SHARD_TRY(outputs(0, rows));
    const auto t1 = std::chrono::steady_clock::now();
    cdb_merge_stats ms{};
    st = merge_device_impl(ctx, &in[0], &o, &out[0], &ms, ctx->stream);
    if (stats) stats[0] = ms;
    X.merge_ms = ms.device_ms;
    X.split_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    X.total_ms = ms_since(t0);
    if (xs) *xs = X;
    return st;
  }

  // ---- 1. owner splits of every source (one synchronisation of every device)
  std::vector<Source> src(N);
  for (int i = 0; i < N; ++i) {
    cdb_ctx* c = slot_ctx(ctx, i);
    const cdb_dev_input& d = in[i];
    Source& S = src[i];
    for (int f = 0; f < 3; ++f) {
      const cdb_dev_rows& r = fam_rows(d, f);
      for (int k = 0; k < kFamCols[f]; ++k) S.cols[f][k] = r.col[k];
      S.stride[f] = std::max<uint32_t>(r.stride, 1);
      if (r.stride0 > 1 || (S.stride[f] > 1 && S.stride[f] != (uint32_t)(kFamCols[f] - 1)))
        return fail(ctx, CDB_BAD_ARGUMENT, "cdb_merge_sharded: input rows must be columns or records");
      if (S.stride[f] != std::max<uint32_t>(fam_rows(in[0], f).stride, 1))
        return fail(ctx, CDB_BAD_ARGUMENT, "cdb_merge_sharded: every device slot's rows must share one layout");
    }
    if (d.keys.n >= (1ull << 32) || d.nodes.n >= (1ull << 32) || d.members.n >= (1ull << 32))
      return fail(ctx, CDB_BAD_ARGUMENT, "row counts must be < 2^32 per family per device");
    if (!runs_valid(d)) continue;
    hipSetDevice(c->device);
    S.R = d.n_runs;
    S.rs.resize(3 * (S.R + 1));
    for (int f = 0; f < 3; ++f)
      for (uint32_t r = 0; r <= S.R; ++r) S.rs[f * (S.R + 1) + r] = d.run_start[f][r];
    S.sp.resize(3ull * S.R * (N + 1));
    uint64_t* w = (uint64_t*)ws_get(c, WS_SPLIT, (S.rs.size() + S.sp.size() + 8) * 8, &st);
    if (!w) return fail_from(c, st);
    SplitArgs a;
    for (int f = 0; f < 3; ++f) {
      a.kh[f] = fam_rows(d, f).col[0];
      a.n[f] = fam_rows(d, f).n;
    }
    a.rs = w;
    a.R = S.R;
    a.world = (uint32_t)N;
    a.bits = bits;
    a.out = w + S.rs.size();
    a.bad = (unsigned long long*)(a.out + S.sp.size());
    hipStream_t s = c->stream;
    CDB_SHARD_HIP(c, hipMemcpyAsync(w, S.rs.data(), S.rs.size() * 8, hipMemcpyHostToDevice, s), "h2d(splits)");
    CDB_SHARD_HIP(c, hipMemsetAsync(a.bad, 0, 8, s), "memset(splits)");
    const uint64_t total = a.n[0] + a.n[1] + a.n[2];
    if (total) run_order_kernel<<<(uint32_t)std::min<uint64_t>((total + 255) / 256, 4096), 256, 0, s>>>(a);
    const uint32_t nt = 3 * S.R * (N + 1);
    owner_split_kernel<<<(nt + 255) / 256, 256, 0, s>>>(a);
    CDB_SHARD_HIP(c, hipGetLastError(), "owner_split_kernel");
    CDB_SHARD_HIP(c, hipMemcpyAsync(S.sp.data(), a.out, S.sp.size() * 8, hipMemcpyDeviceToHost, s), "d2h(splits)");
    CDB_SHARD_HIP(c, hipMemcpyAsync(&S.bad, a.bad, 8, hipMemcpyDeviceToHost, s), "d2h(splits)");
    S.sorted = true;
  }
  for (int i = 0; i < N; ++i) {
    cdb_ctx* c = slot_ctx(ctx, i);
    hipSetDevice(c->device);
    CDB_SHARD_HIP(c, hipStreamSynchronize(c->stream), "sync(splits)");
  }
  // inputs not in runs, or with a run out of order: rows grouped by owner on their device
  for (int i = 0; i < N; ++i) {
    Source& S = src[i];
    if (S.sorted && !S.bad) continue;
    cdb_ctx* c = slot_ctx(ctx, i);
    hipSetDevice(c->device);
    ++X.packed;
    S.sorted = false;
    S.R = 1;
    S.sp.assign(3ull * (N + 1), 0);
    const int slots[3] = {WS_PK, WS_PN, WS_PM};
    for (int f = 0; f < 3; ++f) {
      const cdb_dev_rows& rows = fam_rows(in[i], f);
      cdb_dev_rows packed{};
      CDB_SHARD_TRY(ws_rows(c, slots[f], kFamCols[f], rows.n, S.stride[f], &packed));
      std::vector<uint64_t> cnt(N, 0);
      if (rows.n && (st = cdb_partition_owner(c, &rows, kFamCols[f], bits, &packed, cnt.data(), c->stream)) != CDB_OK)
        return fail_from(c, st);
      for (int k = 0; k < kFamCols[f]; ++k) S.cols[f][k] = packed.col[k];
      uint64_t acc = 0;
      for (int d = 0; d < N; ++d) {
        S.sp[(uint64_t)f * (N + 1) + d] = acc;
        acc += cnt[d];
      }
      S.sp[(uint64_t)f * (N + 1) + N] = acc;
    }
  }
  X.split_ms = ms_since(t0);

  // ---- 2. receive layout of every device: one run per (source, source run) with rows
  struct Recv {
    std::vector<std::pair<int, uint32_t>> runs;
    std::vector<uint64_t> start[3];
    uint64_t total[3] = {0, 0, 0};
    bool sorted = true;
    cdb_dev_rows rows[3];
  };
  uint32_t lay[3];
  for (int f = 0; f < 3; ++f) lay[f] = src[0].stride[f];
  std::vector<Recv> rv(N);
  std::vector<uint32_t> nruns(N);
  uint32_t cap = 0;
  for (int i = 0; i < N; ++i) cap += (nruns[i] = src[i].R);
  for (int d = 0; d < N; ++d) {
    Recv& R = rv[d];
    // the receive layout (cdb_shard_recv_plan, the one plan dist.py uses too): one run per (source,
    // source run) with rows for d, in (source, run) order
    std::vector<uint64_t> counts;
    for (int i = 0; i < N; ++i)
      for (int f = 0; f < 3; ++f)
        for (uint32_t r = 0; r < src[i].R; ++r) counts.push_back(src[i].split(f, r, d + 1, N) - src[i].split(f, r, d, N));
    std::vector<uint32_t> rs(cap + 1), rr(cap + 1);
    std::vector<uint64_t> starts(3ull * (cap + 1));
    uint32_t k = 0;
    if ((st = cdb_shard_recv_plan((uint32_t)N, nruns.data(), counts.data(), cap, &k, rs.data(), rr.data(),
                                  starts.data(), R.total)) != CDB_OK)
      return fail(ctx, st, "cdb_merge_sharded: receive plan");
    for (uint32_t j = 0; j < k; ++j) {
      R.runs.emplace_back((int)rs[j], rr[j]);
      R.sorted = R.sorted && src[rs[j]].sorted;
    }
    for (int f = 0; f < 3; ++f) R.start[f].assign(starts.begin() + f * (cap + 1), starts.begin() + f * (cap + 1) + k + 1);
    cdb_ctx* c = slot_ctx(ctx, d);
    hipSetDevice(c->device);
    const int slots[3] = {WS_XK, WS_XN, WS_XM};
    for (int f = 0; f < 3; ++f) CDB_SHARD_TRY(ws_rows(c, slots[f], kFamCols[f], R.total[f], lay[f], &R.rows[f]));
    CDB_SHARD_TRY(outputs(d, R.total));
  }

  // ---- 3. the exchange: per (source run, family) slice, one transfer per array of the layout
  //         (records: the hash column and the records; columns: every column), in pieces of <= 1 GiB
  const auto t1 = std::chrono::steady_clock::now();
  if (rccl) CDB_SHARD_NCCL(node->group_start(), "ncclGroupStart");
  // an error inside the group still closes it (a group left open would swallow the next call's
  // transfers), and then waits for nothing it posted
  struct GroupGuard {
    const Node* n;
    bool open;
    ~GroupGuard() {
      if (open) n->group_end();
    }
  } guard{node, rccl};
  for (int d = 0; d < N; ++d) {
    const Recv& R = rv[d];
    cdb_ctx* cd = slot_ctx(ctx, d);
    for (size_t k = 0; k < R.runs.size(); ++k) {
      const int i = R.runs[k].first;
      const uint32_t r = R.runs[k].second;
      const Source& S = src[i];
      cdb_ctx* ci = slot_ctx(ctx, i);
      for (int f = 0; f < 3; ++f) {
        const uint64_t a = S.split(f, r, d, N), e = S.split(f, r, d + 1, N);
        if (e == a) continue;
        const uint64_t bytes = (e - a) * 8 * kFamCols[f];
        if (i == d) X.bytes_local += bytes;
        else {
          X.bytes_moved += bytes;
          X.link_bytes[i][d] += bytes;
        }
        for (int col = 0; col < fam_arrays(f, lay[f]); ++col) {
          const uint64_t w = array_words(col, lay[f]);
          const uint64_t* from = S.cols[f][col] + a * w;
          uint64_t* to = R.rows[f].col[col] + R.start[f][k] * w;
          const uint64_t words = (e - a) * w;
          if (i == d || !rccl) {
            hipSetDevice(cd->device);
            const hipError_t e2 = i == d || ci->device == cd->device
                                      ? hipMemcpyAsync(to, from, words * 8, hipMemcpyDeviceToDevice, cd->stream)
                                      : hipMemcpyPeerAsync(to, cd->device, from, ci->device, words * 8, cd->stream);
            CDB_SHARD_HIP(cd, e2, "exchange copy");
            ++X.transfers;
            continue;
          }
          for (uint64_t x = 0; x < words; x += kMaxPieceRows) {
            const uint64_t cnt = std::min<uint64_t>(kMaxPieceRows, words - x);
            hipSetDevice(ci->device);
            CDB_SHARD_NCCL(node->send(from + x, cnt, ncclUint64, d, node->comms[i], ci->stream), "ncclSend");
            hipSetDevice(cd->device);
            CDB_SHARD_NCCL(node->recv(to + x, cnt, ncclUint64, i, node->comms[d], cd->stream), "ncclRecv");
            ++X.transfers;
          }
        }
      }
    }
  }
  if (rccl) {
    guard.open = false;
    CDB_SHARD_NCCL(node->group_end(), "ncclGroupEnd");
  }
  // Wait with a deadline: a transfer that never completes (a peer that never posts its side, a
  // link down) is reported instead of hanging the caller. The context is unusable afterwards.
  const double deadline_ms = 60e3 + (double)(X.bytes_moved + X.bytes_local) / 1e6;  // + 1 ms per MB
  for (int d = 0; d < N; ++d) {
    cdb_ctx* c = slot_ctx(ctx, d);
    hipSetDevice(c->device);
    for (;;) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) CDB_SHARD_HIP(c, q, "sync(exchange)");
      if (ms_since(t1) > deadline_ms)
        return fail(ctx, CDB_DEVICE_ERROR, "cdb_merge_sharded: the row exchange did not complete within " +
                                               std::to_string((long long)deadline_ms) + " ms (device slot " +
                                               std::to_string(d) + ")");
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  X.exchange_ms = ms_since(t1);

  // ---- 4. every device merges what it owns, on its own host thread
  std::vector<cdb_status> rc(N, CDB_OK);
  std::vector<cdb_merge_stats> ms(N);
  auto merge_one = [&](int d) {
    cdb_ctx* c = slot_ctx(ctx, d);
    hipSetDevice(c->device);
    const Recv& R = rv[d];
    cdb_dev_input din;
    std::memset(&din, 0, sizeof din);
    cdb_dev_rows* fam[3] = {&din.keys, &din.nodes, &din.members};
    for (int f = 0; f < 3; ++f) {
      *fam[f] = R.rows[f];
      fam[f]->n = R.total[f];
    }
    din.n_pos = n_pos;
    if (R.sorted && !R.runs.empty() && R.runs.size() <= CDB_MAX_RUNS) {
      din.n_runs = (uint32_t)R.runs.size();
      for (int f = 0; f < 3; ++f)
        for (size_t k = 0; k <= R.runs.size(); ++k) din.run_start[f][k] = R.start[f][k];
    }
    std::memset(&ms[d], 0, sizeof ms[d]);
    rc[d] = merge_device_impl(c, &din, &o, &out[d], &ms[d], c->stream);
  };
  std::vector<std::thread> th;
  for (int d = 1; d < N; ++d) th.emplace_back(merge_one, d);
  merge_one(0);
  for (auto& t : th) t.join();
  for (int d = 0; d < N; ++d) {
    if (stats) stats[d] = ms[d];
    X.merge_ms = std::max(X.merge_ms, ms[d].device_ms);
    if (rc[d] != CDB_OK && st == CDB_OK) st = fail_from(slot_ctx(ctx, d), rc[d]);
  }
  X.total_ms = ms_since(t0);
  if (xs) *xs = X;
  return st;
}

}  // extern "C"
