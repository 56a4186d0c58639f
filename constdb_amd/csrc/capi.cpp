// Host-level C-ABI: decoded batches, the high-level merge (upload, device pipeline,
// download) and the canonical dump of a merge result.
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "batch.h"
#include "engine.h"
#include "ops.h"

namespace cdb {
cdb_status encode_snapshot_impl(cdb_ctx* ctx, const cdb_merged& m, const cdb_encode_header& hdr, uint8_t** out,
                                size_t* out_len, cdb_encode_stats* stats);
cdb_status encode_device_impl(cdb_ctx* ctx, const cdb_dev_output& dout, const std::vector<Batch*>& inputs,
                              const cdb_encode_header& hdr, uint8_t** out, size_t* out_len, cdb_encode_stats* stats);
cdb_status crc64_gpu_impl(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* crc);
cdb_status merge_device_impl(cdb_ctx* ctx, const cdb_dev_input* in, const cdb_merge_opts* opts,
                             cdb_dev_output* out, cdb_merge_stats* stats, hipStream_t s);
}

struct cdb_batch {
  std::shared_ptr<cdb::Batch> b;
};

struct cdb_ops {  // a decoded replicate stream (op rows + byte arena)
  std::shared_ptr<cdb::Batch> b;
  cdb_ops_info info;
};

namespace cdb {
namespace {

constexpr size_t kStageChunk = size_t(32) << 20;  // bytes per pinned slot
constexpr int kStageSlots = 4;                     // = the size of cdb_ctx::pin_ev

int copy_threads() {
  static const int t = [] {
    const char* e = std::getenv("CDB_COPY_THREADS");
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int v = e ? std::atoi(e) : std::min(16, hw);
    return std::max(1, std::min(64, v));
  }();
  return t;
}

struct Piece {
  char* host;
  char* pin;
  char* dev;
  size_t bytes;
};

// Copies every piece between pageable and pinned memory; the bytes are split in equal ranges
// over the copy threads (page faults of fresh destination pages are taken in parallel too).
void par_copy(const std::vector<Piece>& ps, bool to_pin) {
  size_t total = 0;
  for (const Piece& p : ps) total += p.bytes;
  const int T = (int)std::min<size_t>((size_t)copy_threads(), std::max<size_t>(1, total >> 20));
  auto run = [&](size_t lo, size_t hi) {
    size_t base = 0;
    for (const Piece& p : ps) {
      const size_t a = std::max(lo, base), b = std::min(hi, base + p.bytes);
      if (a < b) {
        if (to_pin) std::memcpy(p.pin + (a - base), p.host + (a - base), b - a);
        else std::memcpy(p.host + (a - base), p.pin + (a - base), b - a);
      }
      base += p.bytes;
    }
  };
  if (T <= 1) {
    run(0, total);
    return;
  }
  const size_t per = (total + T - 1) / T;
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(run, std::min(total, t * per), std::min(total, (t + 1) * per));
  run(0, std::min(total, per));
  for (auto& x : th) x.join();
}

}  // namespace

// The first touch of a fresh result buffer (the staged download) then takes one fault per 2 MB
// instead of one per 4 KB.
void advise_huge(void* p, size_t bytes) {
  constexpr uintptr_t kHuge = uintptr_t(2) << 20;
  const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t b = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kHuge - 1);
  if (b > a) madvise(reinterpret_cast<void*>(a), b - a, MADV_HUGEPAGE);
}

void parallel_copy(void* dst, const void* src, size_t bytes) {
  // callers that already decode in parallel (one thread per snapshot) copy on their own thread
  static std::atomic<int> active{0};
  if (bytes < (size_t(8) << 20) || active.fetch_add(1) > 0) {
    if (bytes >= (size_t(8) << 20)) active.fetch_sub(1);
    std::memcpy(dst, src, bytes);
    return;
  }
  par_copy({Piece{static_cast<char*>(dst), const_cast<char*>(static_cast<const char*>(src)), nullptr, bytes}}, false);
  active.fetch_sub(1);
}

void adopt_raw(Batch* b, const uint8_t* buf, size_t len) {
  b->raw.resize(len);  // default-initialised
  advise_huge(b->raw.data(), len);
  parallel_copy(b->raw.data(), buf, len);
}

cdb_status staged_h2d(cdb_ctx* ctx, void* dev, const void* host, size_t bytes, hipStream_t s) {
  if (!bytes) return CDB_OK;
  if (bytes < (size_t(1) << 20)) return hip_check(ctx, hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s), "h2d");
  const HostSeg g{const_cast<void*>(host), dev, bytes};
  return staged_copy(ctx, &g, 1, true, s);
}

cdb_status staged_d2h(cdb_ctx* ctx, void* host, const void* dev, size_t bytes, hipStream_t s) {
  if (!bytes) return CDB_OK;
  if (bytes < (size_t(1) << 20)) {
    cdb_status st = hip_check(ctx, hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s), "d2h");
    return st != CDB_OK ? st : hip_check(ctx, hipStreamSynchronize(s), "d2h sync");
  }
  const HostSeg g{host, const_cast<void*>(dev), bytes};
  return staged_copy(ctx, &g, 1, false, s);
}

cdb_status staged_copy(cdb_ctx* ctx, const HostSeg* segs, size_t nseg, bool h2d, hipStream_t stream) {
  cdb_status st;
  // one ring per context: the decoder's stage threads may stage side by side (decode_gpu.hip), so
  // a call holds the ring -- its lazy allocation, slot cursor and slot events -- until it is done
  std::lock_guard<std::mutex> ring(ctx->pin_mu);
  if (!ctx->pin) {
    if ((st = hip_check(ctx, hipHostMalloc(&ctx->pin, kStageSlots * kStageChunk, hipHostMallocDefault),
                        "hipHostMalloc(staging)")) != CDB_OK) {
      ctx->pin = nullptr;
      return st;
    }
    for (hipEvent_t& e : ctx->pin_ev) {  // created recorded, so the first waits return at once
      if ((st = hip_check(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming), "event")) != CDB_OK) return st;
      if ((st = hip_check(ctx, hipEventRecord(e, stream), "event")) != CDB_OK) return st;
    }
  }
  // chunk jobs: job j fills pinned slot (base + j) % kStageSlots with pieces of one or more
  // segments; the ring continues where the previous call left it
  const uint64_t base = ctx->pin_next;
  std::vector<std::vector<Piece>> jobs;
  std::vector<Piece> cur;
  size_t fill = 0;
  for (size_t i = 0; i < nseg; ++i) {
    for (size_t off = 0; off < segs[i].bytes;) {
      const size_t take = std::min(segs[i].bytes - off, kStageChunk - fill);
      char* slot = static_cast<char*>(ctx->pin) + ((base + jobs.size()) % kStageSlots) * kStageChunk;
      cur.push_back({static_cast<char*>(segs[i].host) + off, slot + fill, static_cast<char*>(segs[i].dev) + off, take});
      fill += take;
      off += take;
      if (fill == kStageChunk) {
        jobs.push_back(std::move(cur));
        cur.clear();
        fill = 0;
      }
    }
  }
  if (!cur.empty()) jobs.push_back(std::move(cur));
  ctx->pin_next = base + jobs.size();
  auto ev_of = [&](size_t j) { return ctx->pin_ev[(base + j) % kStageSlots]; };
  const hipMemcpyKind kind = h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
  // a slot is reused only after the copy recorded on its event (this call's or an earlier one's)
  auto dma = [&](size_t j) -> cdb_status {
    hipEvent_t ev = ev_of(j);
    for (const Piece& p : jobs[j]) {
      void* dst = h2d ? (void*)p.dev : (void*)p.pin;
      const void* src = h2d ? (const void*)p.pin : (const void*)p.dev;
      cdb_status s2 = hip_check(ctx, hipMemcpyAsync(dst, src, p.bytes, kind, stream), "staged copy");
      if (s2 != CDB_OK) return s2;
    }
    return hip_check(ctx, hipEventRecord(ev, stream), "event");
  };
  if (h2d) {
    for (size_t j = 0; j < jobs.size(); ++j) {
      if ((st = hip_check(ctx, hipEventSynchronize(ev_of(j)), "staging wait")) != CDB_OK) return st;
      par_copy(jobs[j], true);
      if ((st = dma(j)) != CDB_OK) return st;
    }
    return CDB_OK;
  }
  for (size_t j = 0; j < jobs.size() && j < (size_t)kStageSlots; ++j) {
    if ((st = hip_check(ctx, hipEventSynchronize(ev_of(j)), "staging wait")) != CDB_OK) return st;
    if ((st = dma(j)) != CDB_OK) return st;
  }
  for (size_t j = 0; j < jobs.size(); ++j) {
    if ((st = hip_check(ctx, hipEventSynchronize(ev_of(j)), "staging wait")) != CDB_OK) return st;
    par_copy(jobs[j], false);
    if (j + kStageSlots < jobs.size() && (st = dma(j + kStageSlots)) != CDB_OK) return st;
  }
  return CDB_OK;
}

}  // namespace cdb


using namespace cdb;

namespace {

std::string hex(const uint8_t* p, uint64_t n) {
  static const char* d = "0123456789abcdef";
  std::string o(n * 2, '0');
  for (uint64_t i = 0; i < n; ++i) {
    o[2 * i] = d[p[i] >> 4];
    o[2 * i + 1] = d[p[i] & 15];
  }
  return o;
}

}  // namespace

// Copies batches [0, n) into the device columns of `din` (batch i's rows after batch i-1's,
// from row `at[f]` of family f on) through the pinned staging ring and stamps fold position
// pos0 + i into batch i's meta words on the device.
static cdb_status upload_batches(cdb_ctx* ctx, cdb_batch* const* inputs, uint32_t n, cdb_dev_input* din,
                                 const uint64_t* at = nullptr, uint32_t pos0 = 0) {
  for (uint32_t i = 0; i < n; ++i)
    if (inputs[i]->b->rows_on_device) return fail(ctx, CDB_BAD_ARGUMENT, "a batch's rows are already in HBM");
  std::vector<HostSeg> segs;
  auto put = [&](const cdb_dev_rows& r, int c, uint64_t off, const ColVec& v) {
    if (!v.empty()) segs.push_back({const_cast<uint64_t*>(v.data()), r.col[c] + off, v.size() * 8});
  };
  const uint64_t k0 = at ? at[0] : 0, n0 = at ? at[1] : 0, m0 = at ? at[2] : 0;
  uint64_t ok = k0, on = n0, om = m0;
  for (uint32_t i = 0; i < n; ++i) {
    const Batch& b = *inputs[i]->b;
    const ColVec* kc[kKeyCols] = {&b.kh, &b.kf, &b.ct, &b.ut, &b.dt, &b.aux, &b.meta};
    const ColVec* nc[kNodeCols] = {&b.n_pkh, &b.n_pkf, &b.n_node, &b.n_v, &b.n_t, &b.n_meta};
    const ColVec* mc[kMemberCols] = {&b.m_pkh, &b.m_pkf, &b.m_h, &b.m_f, &b.m_t, &b.m_meta};
    for (int c = 0; c < kKeyCols; ++c) put(din->keys, c, ok, *kc[c]);
    for (int c = 0; c < kNodeCols; ++c) put(din->nodes, c, on, *nc[c]);
    for (int c = 0; c < kMemberCols; ++c) put(din->members, c, om, *mc[c]);
    ok += b.n_keys();
    on += b.n_nodes();
    om += b.n_members();
  }
  cdb_status st = staged_copy(ctx, segs.data(), segs.size(), true, ctx->stream);
  ok = k0, on = n0, om = m0;
  for (uint32_t i = 0; i < n && st == CDB_OK; ++i) {
    const Batch& b = *inputs[i]->b;
    if ((st = stamp_pos(ctx, din->keys.col[K_META] + ok, b.n_keys(), pos0 + i, ctx->stream)) != CDB_OK ||
        (st = stamp_pos(ctx, din->nodes.col[C_META] + on, b.n_nodes(), pos0 + i, ctx->stream)) != CDB_OK ||
        (st = stamp_pos(ctx, din->members.col[C_META] + om, b.n_members(), pos0 + i, ctx->stream)) != CDB_OK)
      break;
    ok += b.n_keys();
    on += b.n_nodes();
    om += b.n_members();
  }
  return st;
}

// A host result's rows as fold position 0 of the next merge, at rows [0, n) of each family of
// `din` (cdb_merge_into): the key columns kh kf ct ut dt, win staged into aux and meta, then
// state_rows on the device (pos 0, src = the row, aux = a counter's sum).
static cdb_status upload_state(cdb_ctx* ctx, const cdb_merged& m, cdb_dev_input* din) {
  std::vector<HostSeg> segs;
  auto put = [&](const cdb_dev_rows& r, int c, const ColVec& v) {
    if (!v.empty()) segs.push_back({const_cast<uint64_t*>(v.data()), r.col[c], v.size() * 8});
  };
  const int kmap[kKeyCols] = {O_KH, O_KF, O_CT, O_UT, O_DT, O_WIN, O_META};
  for (int c = 0; c < kKeyCols; ++c) put(din->keys, c, m.k[kmap[c]]);
  for (int c = 0; c < kNodeCols; ++c) put(din->nodes, c, m.nd[c]);
  for (int c = 0; c < kMemberCols; ++c) put(din->members, c, m.mb[c]);
  cdb_status st = staged_copy(ctx, segs.data(), segs.size(), true, ctx->stream);
  if (st == CDB_OK) st = state_rows(ctx, din->keys.col[K_META], din->keys.col[K_AUX], m.k[O_KH].size(), ctx->stream);
  if (st == CDB_OK) st = state_rows(ctx, din->nodes.col[C_META], nullptr, m.nd[0].size(), ctx->stream);
  if (st == CDB_OK) st = state_rows(ctx, din->members.col[C_META], nullptr, m.mb[0].size(), ctx->stream);
  return st;
}

// Downloads a compacted device result into m's host columns through the staging ring.
static cdb_status download_result(cdb_ctx* ctx, const cdb_dev_output& dout, cdb_merged* m) {
  std::vector<HostSeg> dsegs;
  auto down = [&](ColVec* dst, int nc, const cdb_dev_rows& r) {
    for (int c = 0; c < nc; ++c) {
      dst[c].resize(r.n);  // default-initialised: no zero fill
      advise_huge(dst[c].data(), r.n * 8);
      if (r.n) dsegs.push_back({dst[c].data(), r.col[c], r.n * 8});
    }
  };
  down(m->k, kKeyOutCols, dout.keys);
  down(m->nd, kNodeCols, dout.nodes);
  down(m->mb, kMemberCols, dout.members);
  return staged_copy(ctx, dsegs.data(), dsegs.size(), false, ctx->stream);
}

// A result whose fold position 0 was `state` (cdb_merge_into, cdb_merged_from_device with a
// state): its byte references become references into state's inputs, so the result stands on
// one flat input list, state's inputs then the new batches (position p >= 1 -> P0 + p - 1, P0 =
// state's input count). A reference (0, src) names row src of the state, whose own reference of
// the same kind is taken: the key row's meta for key bytes, its win for a Bytes value, a
// member's meta for member and field bytes, a node's meta (the head of its segment).
static void flatten_onto(cdb_merged* m, const cdb_merged& state, uint32_t n_new) {
  const uint64_t P0 = state.inputs.size();
  auto remap = [&](uint64_t ref, const ColVec& state_col, bool keep_tag) -> uint64_t {
    const uint32_t p = meta_pos(ref);
    if (p == 0) {
      const uint64_t w = state_col[meta_src(ref)];
      return keep_tag ? meta_pack(meta_tag(ref), meta_pos(w), meta_src(w)) : meta_order(w);
    }
    return meta_pack(keep_tag ? meta_tag(ref) : 0, (uint32_t)(P0 + p - 1), meta_src(ref));
  };
  const uint64_t nk = m->k[O_KH].size();
  for (uint64_t r = 0; r < nk; ++r) {
    const uint64_t mt = m->k[O_META][r];
    const uint32_t T = meta_tag(mt);
    // a side row's win is its last (pos, src); a Bytes key's win the value's (pos, src); a
    // counter's win is its sum, a set's / dict's 0
    if (T == TAG_BYTES) m->k[O_WIN][r] = remap(m->k[O_WIN][r], state.k[O_WIN], false);
    else if (T == TAG_EXPIRE || T == TAG_DELETE) m->k[O_WIN][r] = remap(m->k[O_WIN][r], state.k[O_META], false);
    m->k[O_META][r] = remap(mt, state.k[O_META], true);
  }
  for (uint64_t r = 0; r < m->nd[0].size(); ++r) m->nd[C_META][r] = remap(m->nd[C_META][r], state.nd[C_META], true);
  for (uint64_t r = 0; r < m->mb[0].size(); ++r) m->mb[C_META][r] = remap(m->mb[C_META][r], state.mb[C_META], true);
  m->inputs = state.inputs;
  (void)n_new;
}

// DB::delete (db.rs:73-76) for every Deletes entry of batch b, in stream order: the garbage list.
static void append_garbage(cdb_merged* m, const Batch& b) {
  for (uint64_t i = 0; i < b.n_keys(); ++i)
    if (meta_tag(b.meta[i]) == TAG_DELETE) m->garbage.push_back({b.kh[i], b.kf[i], b.ct[i]});
}

// DB::gc(tombstone)'s pops (db.rs:82-86): from the back, every entry with t <= tombstone is
// processed; the first with t > tombstone ends the loop, popped and lost. Returns how many
// entries stay (the list's front); *first = the first processed entry.
static size_t gc_stop(const cdb_merged& m, uint64_t tombstone, size_t* first) {
  size_t i = m.garbage.size();
  while (i > 0) {
    --i;
    if (m.garbage[i].t > tombstone) {
      *first = i + 1;
      return i;
    }
  }
  *first = 0;
  return 0;
}

// DB::gc (db.rs:82-119) on a host result: every processed entry (key, t) removes the key's Deletes
// row when its time equals t (`deletes.get(&key) == Some(t)`; a removal is final, so the order of
// the pops does not matter); the garbage list keeps the entries before the stop. (Field garbage is
// never enqueued by the reference: delete_field, db.rs:78-80, is uncalled.)
static uint64_t gc_host(cdb_merged* m, uint64_t tombstone) {
  size_t first = 0;
  const size_t keep = gc_stop(*m, tombstone, &first);
  if (keep == m->garbage.size()) return 0;
  const uint64_t nk = m->k[O_KH].size();
  struct KeyHash {
    size_t operator()(const std::pair<uint64_t, uint64_t>& k) const { return k.first ^ (k.second * 0x9E3779B97F4A7C15ull); }
  };
  std::unordered_map<std::pair<uint64_t, uint64_t>, uint64_t, KeyHash> del_row;
  for (uint64_t r = 0; r < nk; ++r)
    if (meta_tag(m->k[O_META][r]) == TAG_DELETE) del_row[{m->k[O_KH][r], m->k[O_KF][r]}] = r;
  std::vector<uint8_t> drop(nk, 0);
  uint64_t removed = 0;
  for (size_t i = first; i < m->garbage.size(); ++i) {
    const cdb_merged::Garbage& g = m->garbage[i];
    auto it = del_row.find({g.kh, g.kf});
    if (it != del_row.end() && !drop[it->second] && m->k[O_CT][it->second] == g.t) {
      drop[it->second] = 1;
      ++removed;
    }
  }
  m->garbage.resize(keep);
  if (removed) {
    uint64_t w = 0;
    for (uint64_t r = 0; r < nk; ++r) {
      if (drop[r]) continue;
      if (w != r)
        for (int c = 0; c < kKeyOutCols; ++c) m->k[c][w] = m->k[c][r];
      ++w;
    }
    for (int c = 0; c < kKeyOutCols; ++c) m->k[c].resize(w);
  }
  return removed;
}

extern "C" {

cdb_status cdb_decode_snapshot(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags, cdb_batch** out,
                               size_t* err_offset) {
  (void)ctx;
  if (!out || (!buf && len)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  auto b = std::make_shared<Batch>();
  size_t eo = 0;
  const int rc = decode_snapshot(buf, len, flags, b.get(), &eo);
  if (err_offset) *err_offset = eo;
  if (rc == CDB_OK || rc == CDB_INVALID_SNAPSHOT_CHECKSUM) {
    *out = new cdb_batch{b};
  }
  return (cdb_status)rc;
}

cdb_status cdb_decode_snapshot_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint32_t flags, cdb_batch** out,
                                   size_t* err_offset, double* index_ms, double* device_ms) {
  if (!out || (!buf && len)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if (!ctx) return CDB_NO_DEVICE;
  auto b = std::make_shared<Batch>();
  size_t eo = 0;
  DecodeTiming tm;
  const int rc = decode_snapshot_gpu(ctx, buf, len, flags, b.get(), &eo, &tm);
  if (err_offset) *err_offset = eo;
  if (index_ms) *index_ms = tm.index_ms;
  if (device_ms) *device_ms = tm.device_ms;
  if (rc == CDB_OK || rc == CDB_INVALID_SNAPSHOT_CHECKSUM) *out = new cdb_batch{b};
  return (cdb_status)rc;
}

cdb_status cdb_decode_snapshots_device(cdb_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, uint32_t n,
                                       uint32_t flags, cdb_batch** batches, cdb_dev_input* out, uint32_t* failed,
                                       size_t* err_offset, double* index_ms, double* device_ms) {
  if (!batches || !out || (n && (!bufs || !lens))) return CDB_BAD_ARGUMENT;
  if (!ctx) return CDB_NO_DEVICE;
  if (n > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 63 snapshots per merge");
  for (uint32_t i = 0; i < n; ++i) {
    batches[i] = nullptr;
    if (!bufs[i] && lens[i]) return CDB_BAD_ARGUMENT;
  }
  std::vector<std::shared_ptr<Batch>> bs(n);
  std::vector<Batch*> raw(n);
  for (uint32_t i = 0; i < n; ++i) {
    bs[i] = std::make_shared<Batch>();
    raw[i] = bs[i].get();
  }
  uint32_t fi = 0;
  size_t eo = 0;
  DecodeTiming tm;
  hipSetDevice(ctx->device);
  const int rc = decode_snapshots_gpu_device(ctx, bufs, lens, n, flags, raw.data(), out, &fi, &eo, &tm);
  if (failed) *failed = fi;
  if (err_offset) *err_offset = eo;
  if (index_ms) *index_ms = tm.index_ms;
  if (device_ms) *device_ms = tm.device_ms;
  if (rc == CDB_OK || rc == CDB_INVALID_SNAPSHOT_CHECKSUM)
    for (uint32_t i = 0; i < n; ++i) batches[i] = new cdb_batch{bs[i]};
  return (cdb_status)rc;
}

cdb_status cdb_batch_info_get(const cdb_batch* cb, cdb_batch_info* info) {
  if (!cb || !info) return CDB_BAD_ARGUMENT;
  const Batch& b = *cb->b;
  std::memset(info, 0, sizeof *info);
  info->n_data = b.n_data;
  info->n_expires = b.n_expires;
  info->n_deletes = b.n_deletes;
  info->n_nodes = b.rows_on_device ? b.dev_rows[1] : b.n_nodes();
  info->n_members = b.rows_on_device ? b.dev_rows[2] : b.n_members();
  info->node_id = b.node_id;
  info->uuid_he_sent = b.uuid_he_sent;
  info->n_replica_add = (uint32_t)b.replica_add.size();
  info->n_replica_del = (uint32_t)b.replica_del.size();
  std::snprintf(info->version, sizeof info->version, "%s", b.version.c_str());
  return CDB_OK;
}

cdb_status cdb_batch_column(const cdb_batch* cb, int family, int col, const uint64_t** data, uint64_t* n) {
  if (!cb || !data || !n) return CDB_BAD_ARGUMENT;
  const Batch& b = *cb->b;
  if (b.rows_on_device) return CDB_BAD_ARGUMENT;  // its rows are in HBM (cdb_decode_snapshots_device)
  const ColVec* k[] = {&b.kh, &b.kf, &b.ct, &b.ut, &b.dt, &b.aux, &b.meta};
  const ColVec* nd[] = {&b.n_pkh, &b.n_pkf, &b.n_node, &b.n_v, &b.n_t, &b.n_meta};
  const ColVec* mb[] = {&b.m_pkh, &b.m_pkf, &b.m_h, &b.m_f, &b.m_t, &b.m_meta};
  const ColVec* v = nullptr;
  if (family == 0 && col >= 0 && col < kKeyCols) v = k[col];
  else if (family == 1 && col >= 0 && col < kNodeCols) v = nd[col];
  else if (family == 2 && col >= 0 && col < kMemberCols) v = mb[col];
  if (!v) return CDB_BAD_ARGUMENT;
  *data = v->data();
  *n = v->size();
  return CDB_OK;
}

void cdb_batch_free(cdb_batch* b) { delete b; }

cdb_status cdb_merge(cdb_ctx* ctx, cdb_batch* const* inputs, uint32_t n, const cdb_merge_opts* opts, cdb_merged** out,
                     cdb_merge_stats* stats) {
  if (!ctx || !out || (n && !inputs)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if (n > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 63 batches per merge");
  hipSetDevice(ctx->device);
  // batches are folded in array order: pos = array index, stamped into meta below
  uint64_t K = 0, N = 0, M = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!inputs[i] || inputs[i]->b->rows_on_device)
      return fail(ctx, CDB_BAD_ARGUMENT, "cdb_merge: a batch's rows are in HBM; merge them with cdb_merge_device");
  for (uint32_t i = 0; i < n; ++i) {
    K += inputs[i]->b->n_keys();
    N += inputs[i]->b->n_nodes();
    M += inputs[i]->b->n_members();
  }
  // Each batch's columns go straight from its host vectors to their offset in one device
  // column per field (no host-side concatenation); the fold position is stamped into the meta
  // words on the device. Input and output blocks are context workspace, reused across calls.
  const bool timing = std::getenv("CDB_HOST_TIMING") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  cdb_dev_input din;
  std::memset(&din, 0, sizeof din);
  cdb_dev_output dout;
  std::memset(&dout, 0, sizeof dout);
  din.n_pos = n;
  cdb_status st = CDB_OK;
  auto block = [&](int slot, int ncol, uint64_t rows, cdb_dev_rows* r) -> cdb_status {
    const uint64_t cap = std::max<uint64_t>(rows, 1);
    auto* p = static_cast<uint64_t*>(ws_get(ctx, slot, ncol * cap * 8, &st));
    if (!p) return st;
    std::memset(r, 0, sizeof *r);
    for (int c = 0; c < ncol; ++c) r->col[c] = p + c * cap;
    r->n = rows;
    return CDB_OK;
  };
  if ((st = block(WS_HOST_IN_K, kKeyCols, K, &din.keys)) != CDB_OK ||
      (st = block(WS_HOST_IN_N, kNodeCols, N, &din.nodes)) != CDB_OK ||
      (st = block(WS_HOST_IN_M, kMemberCols, M, &din.members)) != CDB_OK ||
      (st = block(WS_HOST_OUT_K, kKeyOutCols, K, &dout.keys)) != CDB_OK ||
      (st = block(WS_HOST_OUT_N, kNodeCols, N, &dout.nodes)) != CDB_OK ||
      (st = block(WS_HOST_OUT_M, kMemberCols, M, &dout.members)) != CDB_OK)
    return st;
  if ((st = upload_batches(ctx, inputs, n, &din)) != CDB_OK) return st;
  const auto t1 = std::chrono::steady_clock::now();
  dout.compact = 1;
  cdb_merge_stats local;
  st = merge_device_impl(ctx, &din, opts, &dout, stats ? stats : &local, ctx->stream);
  if (st != CDB_OK && st != CDB_DICT_MERGE_UNIMPLEMENTED) return st;
  const cdb_status merge_st = st;
  const auto t2 = std::chrono::steady_clock::now();
  auto* m = new cdb_merged();
  for (uint32_t i = 0; i < n; ++i) m->inputs.push_back(inputs[i]->b);
  if ((st = download_result(ctx, dout, m)) != CDB_OK) {
    delete m;
    return st;
  }
  // the garbage list: this merge's Deletes entries in fold order; with DB::gc in the merge (the
  // kernels applied its rule to the same list) the entries the pops took are gone
  for (uint32_t i = 0; i < n; ++i) append_garbage(m, *inputs[i]->b);
  if (opts && (opts->flags & CDB_MERGE_GC_DELETES)) {
    size_t first = 0;
    m->garbage.resize(gc_stop(*m, opts->gc_watermark, &first));
  }
  if (timing) {
    const auto t3 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::fprintf(stderr, "cdb_merge host timing: upload %.1f ms, merge %.1f ms, download %.1f ms\n", ms(t0, t1),
                 ms(t1, t2), ms(t2, t3));
  }
  *out = m;
  return merge_st;
}

cdb_status cdb_upload_batches(cdb_ctx* ctx, cdb_batch* const* inputs, uint32_t n, cdb_dev_input* out) {
  if (!ctx || !out || (n && !inputs)) return CDB_BAD_ARGUMENT;
  std::memset(out, 0, sizeof *out);
  if (n > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 63 batches per merge");
  hipSetDevice(ctx->device);
  uint64_t K = 0, N = 0, M = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!inputs[i] || inputs[i]->b->rows_on_device)
      return fail(ctx, CDB_BAD_ARGUMENT, "cdb_merge: a batch's rows are in HBM; merge them with cdb_merge_device");
  for (uint32_t i = 0; i < n; ++i) {
    K += inputs[i]->b->n_keys();
    N += inputs[i]->b->n_nodes();
    M += inputs[i]->b->n_members();
  }
  cdb_status st;
  if ((st = cdb_dev_rows_alloc(ctx, &out->keys, K, kKeyCols)) != CDB_OK ||
      (st = cdb_dev_rows_alloc(ctx, &out->nodes, N, kNodeCols)) != CDB_OK ||
      (st = cdb_dev_rows_alloc(ctx, &out->members, M, kMemberCols)) != CDB_OK ||
      (st = upload_batches(ctx, inputs, n, out)) != CDB_OK ||
      (st = hip_check(ctx, hipStreamSynchronize(ctx->stream), "upload")) != CDB_OK) {
    cdb_dev_rows_release(ctx, &out->keys);
    cdb_dev_rows_release(ctx, &out->nodes);
    cdb_dev_rows_release(ctx, &out->members);
    return st;
  }
  out->n_pos = n;
  return CDB_OK;
}

cdb_status cdb_merge_into(cdb_ctx* ctx, cdb_merged* state, cdb_batch* const* inputs, uint32_t n,
                          const cdb_merge_opts* opts, cdb_merged** out, cdb_merge_stats* stats) {
  if (!ctx || !state || !out || (n && !inputs)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if (n + 1 > (uint32_t)kMaxPos) return fail(ctx, CDB_BAD_ARGUMENT, "at most 62 batches merged into a state");
  if (state->inputs.size() + n > 255) return fail(ctx, CDB_BAD_ARGUMENT, "at most 255 inputs behind one result");
  for (uint32_t i = 0; i < n; ++i)
    if (!inputs[i] || inputs[i]->b->rows_on_device)
      return fail(ctx, CDB_BAD_ARGUMENT, "cdb_merge_into: a batch's rows are in HBM; merge them with cdb_merge_device");
  hipSetDevice(ctx->device);
  const uint64_t sk = state->k[O_KH].size(), sn = state->nd[0].size(), sm = state->mb[0].size();
  uint64_t K = sk, N = sn, M = sm;
  for (uint32_t i = 0; i < n; ++i) {
    K += inputs[i]->b->n_keys();
    N += inputs[i]->b->n_nodes();
    M += inputs[i]->b->n_members();
  }
  cdb_dev_input din;
  std::memset(&din, 0, sizeof din);
  cdb_dev_output dout;
  std::memset(&dout, 0, sizeof dout);
  din.n_pos = n + 1;
  cdb_status st = CDB_OK;
  auto block = [&](int slot, int ncol, uint64_t rows, cdb_dev_rows* r) -> cdb_status {
    const uint64_t cap = std::max<uint64_t>(rows, 1);
    auto* p = static_cast<uint64_t*>(ws_get(ctx, slot, ncol * cap * 8, &st));
    if (!p) return st;
    std::memset(r, 0, sizeof *r);
    for (int c = 0; c < ncol; ++c) r->col[c] = p + c * cap;
    r->n = rows;
    return CDB_OK;
  };
  if ((st = block(WS_HOST_IN_K, kKeyCols, K, &din.keys)) != CDB_OK ||
      (st = block(WS_HOST_IN_N, kNodeCols, N, &din.nodes)) != CDB_OK ||
      (st = block(WS_HOST_IN_M, kMemberCols, M, &din.members)) != CDB_OK ||
      (st = block(WS_HOST_OUT_K, kKeyOutCols, K, &dout.keys)) != CDB_OK ||
      (st = block(WS_HOST_OUT_N, kNodeCols, N, &dout.nodes)) != CDB_OK ||
      (st = block(WS_HOST_OUT_M, kMemberCols, M, &dout.members)) != CDB_OK)
    return st;
  const uint64_t at[3] = {sk, sn, sm};
  if ((st = upload_state(ctx, *state, &din)) != CDB_OK) return st;
  if ((st = upload_batches(ctx, inputs, n, &din, at, 1)) != CDB_OK) return st;
  dout.compact = 1;
  // DB::gc after a chain pops the state's garbage list, not only this merge's entries (the state's
  // Deletes rows are its deletes map, not its list): the device merge runs without it, and the
  // gc runs on the result over state.garbage ++ the new entries (gc_host)
  cdb_merge_opts o;
  std::memset(&o, 0, sizeof o);
  if (opts) o = *opts;
  const bool gc = (o.flags & CDB_MERGE_GC_DELETES) != 0;
  o.flags &= ~(uint32_t)CDB_MERGE_GC_DELETES;
  cdb_merge_stats local;
  cdb_merge_stats* ms = stats ? stats : &local;
  st = merge_device_impl(ctx, &din, &o, &dout, ms, ctx->stream);
  if (st != CDB_OK && st != CDB_DICT_MERGE_UNIMPLEMENTED) return st;
  const cdb_status merge_st = st;
  auto m = std::make_unique<cdb_merged>();
  if ((st = download_result(ctx, dout, m.get())) != CDB_OK) return st;
  flatten_onto(m.get(), *state, n);
  for (uint32_t i = 0; i < n; ++i) m->inputs.push_back(inputs[i]->b);
  m->garbage = state->garbage;
  for (uint32_t i = 0; i < n; ++i) append_garbage(m.get(), *inputs[i]->b);
  if (gc) {
    const uint64_t removed = gc_host(m.get(), o.gc_watermark);
    ms->deletes_gced = removed;
    ms->key_rows_out -= removed;
  }
  *out = m.release();
  return merge_st;
}

cdb_status cdb_merged_from_device(cdb_ctx* ctx, cdb_merged* state, cdb_batch* const* inputs, uint32_t n,
                                  const cdb_dev_output* dout, cdb_merged** out) {
  if (!ctx || !dout || !out || (n && !inputs)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if ((state ? state->inputs.size() : 0) + n > 255) return fail(ctx, CDB_BAD_ARGUMENT, "at most 255 inputs behind one result");
  for (uint32_t i = 0; i < n; ++i)
    if (!inputs[i]) return CDB_BAD_ARGUMENT;
  hipSetDevice(ctx->device);
  auto m = std::make_unique<cdb_merged>();
  cdb_status st = CDB_OK;
  if (dout->compact) {
    st = download_result(ctx, *dout, m.get());
  } else {  // the bucket layout: compacted into temporary columns first
    cdb_dev_output dense;
    std::memset(&dense, 0, sizeof dense);
    st = cdb_dev_rows_alloc(ctx, &dense.keys, dout->keys.n, kKeyOutCols);
    if (st == CDB_OK) st = cdb_dev_rows_alloc(ctx, &dense.nodes, dout->nodes.n, kNodeCols);
    if (st == CDB_OK) st = cdb_dev_rows_alloc(ctx, &dense.members, dout->members.n, kMemberCols);
    if (st == CDB_OK) st = cdb_dev_output_compact(ctx, dout, &dense, nullptr);
    if (st == CDB_OK) st = download_result(ctx, dense, m.get());
    cdb_dev_rows_release(ctx, &dense.keys);
    cdb_dev_rows_release(ctx, &dense.nodes);
    cdb_dev_rows_release(ctx, &dense.members);
  }
  if (st != CDB_OK) return st;
  if (state) flatten_onto(m.get(), *state, n);
  for (uint32_t i = 0; i < n; ++i) m->inputs.push_back(inputs[i]->b);
  // (the garbage list: state's, then the host-resident batches' entries; a batch decoded into HBM
  // keeps its rows there, so a result over such batches starts no list -- see cdb_merged_gc)
  if (state) m->garbage = state->garbage;
  for (uint32_t i = 0; i < n; ++i)
    if (!inputs[i]->b->rows_on_device) append_garbage(m.get(), *inputs[i]->b);
  *out = m.release();
  return CDB_OK;
}

cdb_status cdb_merged_gc(cdb_ctx* ctx, cdb_merged* m, uint64_t tombstone, uint64_t* removed) {
  (void)ctx;
  if (!m) return CDB_BAD_ARGUMENT;
  const uint64_t r = gc_host(m, tombstone);
  if (removed) *removed = r;
  return CDB_OK;
}

uint64_t cdb_merged_garbage_count(const cdb_merged* m) { return m ? m->garbage.size() : 0; }

cdb_status cdb_merged_canonical_dump(cdb_ctx* ctx, cdb_merged* m, char** out, size_t* len) {
  if (!m || !out || !len) return CDB_BAD_ARGUMENT;
  for (const auto& b : m->inputs)  // (byte references a device decode left in HBM)
    if (cdb_status st = refs_ready(ctx, b.get()); st != CDB_OK) return st;
  const uint64_t nk = m->k[O_KH].size();
  struct KeyView { const uint8_t* p; uint64_t n; uint64_t row; };
  auto key_of = [&](uint64_t r) {
    const uint64_t mt = m->k[O_META][r];
    const Batch& b = *m->inputs[meta_pos(mt)];
    const ByteRef kr = b.key_ref[meta_src(mt)];
    return KeyView{b.raw.data() + kr.off, kr.len, r};
  };
  auto less = [](const KeyView& a, const KeyView& b) {
    const int c = std::memcmp(a.p, b.p, std::min(a.n, b.n));
    return c != 0 ? c < 0 : a.n < b.n;
  };
  std::vector<KeyView> data, exps, dels;
  for (uint64_t r = 0; r < nk; ++r) {
    const uint32_t T = meta_tag(m->k[O_META][r]);
    (T == TAG_EXPIRE ? exps : T == TAG_DELETE ? dels : data).push_back(key_of(r));
  }
  std::sort(data.begin(), data.end(), less);
  std::sort(exps.begin(), exps.end(), less);
  std::sort(dels.begin(), dels.end(), less);
  std::string o;
  char buf[160];
  for (const KeyView& kv : data) {
    const uint64_t r = kv.row;
    const uint32_t T = meta_tag(m->k[O_META][r]);
    std::snprintf(buf, sizeof buf, " %u %llu %llu %llu\n", T, (unsigned long long)m->k[O_CT][r],
                  (unsigned long long)m->k[O_UT][r], (unsigned long long)m->k[O_DT][r]);
    o += "K " + hex(kv.p, kv.n) + buf;
    const uint64_t cref = m->k[O_CREF][r];
    const uint64_t cb = cref >> 24, cc = cref & 0xFFFFFF;
    if (T == TAG_BYTES) {
      const uint64_t w = m->k[O_WIN][r];
      const Batch& b = *m->inputs[meta_pos(w)];
      const ByteRef v = b.val_ref[meta_src(w)];
      o += " V " + hex(b.raw.data() + v.off, v.len) + "\n";
    } else if (T == TAG_COUNTER) {
      std::snprintf(buf, sizeof buf, " S %lld\n", (long long)m->k[O_WIN][r]);
      o += buf;
      std::vector<uint64_t> rows;
      for (uint64_t j = cb; j < cb + cc; ++j) rows.push_back(j);
      std::sort(rows.begin(), rows.end(), [&](uint64_t a, uint64_t b) { return m->nd[C_ID1][a] < m->nd[C_ID1][b]; });
      for (uint64_t j : rows) {
        std::snprintf(buf, sizeof buf, " N %llu %lld %llu\n", (unsigned long long)m->nd[C_ID1][j],
                      (long long)m->nd[C_ID2][j], (unsigned long long)m->nd[C_T][j]);
        o += buf;
      }
    } else {
      struct MV { const uint8_t* p; uint64_t n; uint64_t row; };
      std::vector<MV> ms;
      for (uint64_t j = cb; j < cb + cc; ++j) {
        const uint64_t mt = m->mb[C_META][j];
        const Batch& b = *m->inputs[meta_pos(mt)];
        const ByteRef mr = b.m_ref[meta_src(mt)];
        ms.push_back(MV{b.raw.data() + mr.off, mr.len, j});
      }
      std::sort(ms.begin(), ms.end(), [](const MV& a, const MV& b) {
        const int c = std::memcmp(a.p, b.p, std::min(a.n, b.n));
        return c != 0 ? c < 0 : a.n < b.n;
      });
      for (const MV& mv : ms) {
        const uint64_t mt = m->mb[C_META][mv.row];
        std::snprintf(buf, sizeof buf, " %llu", (unsigned long long)m->mb[C_T][mv.row]);
        if (meta_tag(mt) == KIND_ADD) {
          o += " A " + hex(mv.p, mv.n) + buf;
          if (T == TAG_DICT) {
            const Batch& b = *m->inputs[meta_pos(mt)];
            const ByteRef vr = b.m_vref[meta_src(mt)];
            o += " " + hex(b.raw.data() + vr.off, vr.len);
          }
          o += "\n";
        } else {
          o += " D " + hex(mv.p, mv.n) + buf + "\n";
        }
      }
    }
  }
  for (int side = 0; side < 2; ++side) {
    for (const KeyView& kv : side == 0 ? exps : dels) {
      std::snprintf(buf, sizeof buf, " %llu\n", (unsigned long long)m->k[O_CT][kv.row]);
      o += std::string(side == 0 ? "X " : "R ") + hex(kv.p, kv.n) + buf;
    }
  }
  *out = (char*)std::malloc(o.size() + 1);
  if (!*out) return CDB_OUT_OF_MEMORY;
  std::memcpy(*out, o.data(), o.size());
  (*out)[o.size()] = 0;
  *len = o.size();
  return CDB_OK;
}

// Replica-metadata merge (replica/pull.rs:131-156): ReplicaManager::add_replica / remove_replica
// over LWWHash<addr, ReplicaMeta> (replica/replica.rs:29-35, crdt/lwwhash.rs:87-128).
cdb_status cdb_merged_replicas(cdb_merged* m, const cdb_replica_entry** out, size_t* n) {
  if (!m || !out || !n) return CDB_BAD_ARGUMENT;
  if (!m->replicas_done) {
    struct Add { uint64_t t, id, uuid; std::string alias; };
    std::map<std::string, Add> add;        // addr -> (add_time, meta)
    std::map<std::string, uint64_t> del;   // addr -> del_time
    auto set = [&](const std::string& k, const Add& v) {  // lwwhash.rs:87-107
      auto d = del.find(k);
      if (d != del.end() && d->second > v.t) return;
      auto a = add.find(k);
      if (a != add.end()) {
        if (a->second.t > v.t) return;
        a->second = v;
      } else {
        if (d != del.end()) del.erase(d);
        add.emplace(k, v);
      }
    };
    auto rem = [&](const std::string& k, uint64_t t) {  // lwwhash.rs:109-128
      auto a = add.find(k);
      if (a != add.end() && a->second.t > t) return;
      auto d = del.find(k);
      if (d != del.end()) {
        if (d->second > t) return;
        d->second = t;
      } else {
        del.emplace(k, t);
        if (a != add.end()) add.erase(a);
      }
    };
    const uint64_t myself = m->inputs.empty() ? 0 : m->inputs[0]->node_id;
    for (size_t i = 0; i < m->inputs.size(); ++i) {
      const Batch& b = *m->inputs[i];
      if (i == 0) {  // the local ReplicaManager itself: its maps as dumped (replica.rs:100-119)
        for (const ReplicaAdd& r : b.replica_add) add[r.addr] = Add{r.add_time, r.node_id, r.uuid, r.alias};
        for (const ReplicaDel& r : b.replica_del) del[r.addr] = r.t;
        continue;
      }
      size_t ia = 0, id = 0;  // the two lists merged back into stream order
      while (ia < b.replica_add.size() || id < b.replica_del.size()) {
        const bool take_add =
            id == b.replica_del.size() || (ia < b.replica_add.size() && b.replica_add[ia].seq < b.replica_del[id].seq);
        if (take_add) {
          const ReplicaAdd& r = b.replica_add[ia++];
          if (r.node_id != myself) set(r.addr, Add{r.add_time, r.node_id, r.uuid, r.alias});  // pull.rs:133-135
        } else {
          const ReplicaDel& r = b.replica_del[id++];
          rem(r.addr, r.t);
        }
      }
    }
    std::map<std::string, cdb_replica_entry> all;
    m->rep_str.reserve(2 * (add.size() + del.size()) + 1);
    auto keep = [&](const std::string& x) {
      m->rep_str.push_back(x);
      return m->rep_str.back().c_str();
    };
    for (auto& kv : add) {
      cdb_replica_entry e{};
      e.addr = keep(kv.first);
      e.alias = keep(kv.second.alias);
      e.node_id = kv.second.id;
      e.uuid_he_sent = kv.second.uuid;
      e.add_time = kv.second.t;
      e.has_add = 1;
      all[kv.first] = e;
    }
    for (auto& kv : del) {
      auto it = all.find(kv.first);
      if (it == all.end()) {
        cdb_replica_entry e{};
        e.addr = keep(kv.first);
        e.alias = keep("");
        it = all.emplace(kv.first, e).first;
      }
      it->second.del_time = kv.second;
      it->second.has_del = 1;
    }
    for (auto& kv : all) m->replicas.push_back(kv.second);
    m->replicas_done = true;
  }
  *out = m->replicas.empty() ? nullptr : m->replicas.data();
  *n = m->replicas.size();
  return CDB_OK;
}

cdb_status cdb_decode_ops(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, cdb_ops** out,
                          size_t* err_offset) {
  (void)ctx;
  if (!out || (!buf && len)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  auto o = std::make_unique<cdb_ops>();
  o->b = std::make_shared<Batch>();
  size_t eo = 0;
  const int rc = decode_ops(buf, len, uuid_he_sent, o->b.get(), &o->info, &eo);
  if (err_offset) *err_offset = eo;
  if (rc == CDB_OK || rc == CDB_NEED_MORE_MSG) *out = o.release();
  return (cdb_status)rc;
}

cdb_status cdb_decode_ops_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t uuid_he_sent, cdb_ops** out,
                              size_t* err_offset, double* host_ms, double* device_ms, uint32_t* used_gpu) {
  if (!ctx || !out || (!buf && len)) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  if (host_ms) *host_ms = 0;
  if (device_ms) *device_ms = 0;
  if (used_gpu) *used_gpu = 1;
  auto o = std::make_unique<cdb_ops>();
  o->b = std::make_shared<Batch>();
  size_t eo = 0;
  int rc = CDB_OK;
  const int g = decode_ops_gpu(ctx, buf, len, uuid_he_sent, o->b.get(), &o->info, &eo, &rc, host_ms, device_ms);
  if (g < 0) return (cdb_status)(-g);  // a device fault or out of memory: reported, not masked
  if (g != 0) {
    // a shape the device path leaves to the host decoder: the whole stream goes there
    (void)hipGetLastError();
    if (used_gpu) *used_gpu = 0;
    o->b = std::make_shared<Batch>();
    const auto t0 = std::chrono::steady_clock::now();
    rc = decode_ops(buf, len, uuid_he_sent, o->b.get(), &o->info, &eo);
    if (host_ms) *host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  if (err_offset) *err_offset = eo;
  if (rc == CDB_OK || rc == CDB_NEED_MORE_MSG) *out = o.release();
  return (cdb_status)rc;
}

cdb_status cdb_snapshot_index_selftest(const uint8_t* buf, size_t len, uint32_t flags, uint32_t threads,
                                       uint64_t* entries) {
  Batch b1, b2;
  EntryIndex i1, i2;
  DeferredCrc c1, c2;
  size_t e1 = 0, e2 = 0;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const int r1 = index_snapshot(buf, len, flags, &b1, &i1, &e1, &c1, 1);
  const auto t1 = clk::now();
  const int r2 = index_snapshot(buf, len, flags, &b2, &i2, &e2, &c2, threads);
  const auto t2 = clk::now();
  if (std::getenv("CDB_SELFTEST_TIMING")) {
    Batch b3;
    const auto t3 = clk::now();
    adopt_raw(&b3, buf, len);
    const auto t4 = clk::now();
    fprintf(stderr, "index: sequential %.1f ms, %u threads %.1f ms, of which the arena copy %.1f ms\n",
            std::chrono::duration<double, std::milli>(t1 - t0).count(), threads,
            std::chrono::duration<double, std::milli>(t2 - t1).count(),
            std::chrono::duration<double, std::milli>(t4 - t3).count());
  }
  if (entries) *entries = i1.offset.size();
  const bool same = r1 == r2 && e1 == e2 && i1.offset == i2.offset && i1.kind == i2.kind && c1.pending == c2.pending &&
                    c1.len == c2.len && c1.got == c2.got && c1.err_off == c2.err_off && b1.n_data == b2.n_data &&
                    b1.n_expires == b2.n_expires && b1.n_deletes == b2.n_deletes;
  if (!same && std::getenv("CDB_SELFTEST_VERBOSE")) {
    size_t k = 0;
    while (k < i1.offset.size() && k < i2.offset.size() && i1.offset[k] == i2.offset[k] && i1.kind[k] == i2.kind[k]) ++k;
    fprintf(stderr, "selftest: rc %d/%d err %zu/%zu entries %zu/%zu first diff %zu (%llu/%llu) data %llu/%llu crc %d/%d %llu/%llu\n",
            r1, r2, e1, e2, i1.offset.size(), i2.offset.size(), k,
            (unsigned long long)(k < i1.offset.size() ? i1.offset[k] : 0), (unsigned long long)(k < i2.offset.size() ? i2.offset[k] : 0),
            (unsigned long long)b1.n_data, (unsigned long long)b2.n_data, (int)c1.pending, (int)c2.pending,
            (unsigned long long)c1.len, (unsigned long long)c2.len);
  }
  return same ? CDB_OK : CDB_DEVICE_ERROR;
}

cdb_status cdb_ops_column(const cdb_ops* ops, int family, int col, const uint64_t** data, uint64_t* n) {
  if (!ops || !data || !n) return CDB_BAD_ARGUMENT;
  const Batch& b = *ops->b;
  const ColVec* k[] = {&b.kh, &b.kf, &b.ct, &b.ut, &b.dt, &b.aux, &b.meta};
  const ColVec* nd[] = {&b.n_pkh, &b.n_pkf, &b.n_node, &b.n_v, &b.n_t, &b.n_meta};
  const ColVec* mb[] = {&b.m_pkh, &b.m_pkf, &b.m_h, &b.m_f, &b.m_t, &b.m_meta};
  const RefVec* r = nullptr;
  const ColVec* v = nullptr;
  if (family == 0 && col >= 0 && col < kKeyCols) v = k[col];
  else if (family == 0 && col == kKeyCols) r = &b.key_ref;
  else if (family == 0 && col == kKeyCols + 1) r = &b.val_ref;
  else if (family == 1 && col >= 0 && col < kNodeCols) v = nd[col];
  else if (family == 2 && col >= 0 && col < kMemberCols) v = mb[col];
  else if (family == 2 && col == kMemberCols) r = &b.m_ref;
  else if (family == 2 && col == kMemberCols + 1) r = &b.m_vref;
  if (v) {
    *data = v->data();
    *n = v->size();
    return CDB_OK;
  }
  if (r) {
    static_assert(sizeof(ByteRef) == 16, "(offset, length) pairs");
    *data = reinterpret_cast<const uint64_t*>(r->data());
    *n = 2 * r->size();
    return CDB_OK;
  }
  return CDB_BAD_ARGUMENT;
}

cdb_status cdb_ops_info_get(const cdb_ops* ops, cdb_ops_info* info) {
  if (!ops || !info) return CDB_BAD_ARGUMENT;
  *info = ops->info;
  return CDB_OK;
}

void cdb_ops_free(cdb_ops* ops) { delete ops; }

cdb_status cdb_apply_ops(cdb_ctx* ctx, cdb_merged* state, const cdb_ops* ops, cdb_merged** out,
                         cdb_apply_stats* stats) {
  if (!ctx || !state || !ops || !out) return CDB_BAD_ARGUMENT;
  *out = nullptr;
  const uint32_t pos = (uint32_t)state->inputs.size();
  if (pos >= 255) return fail(ctx, CDB_BAD_ARGUMENT, "at most 255 fold positions per result");
  hipSetDevice(ctx->device);
  auto m = std::make_unique<cdb_merged>();
  m->inputs = state->inputs;
  m->inputs.push_back(ops->b);
  m->garbage = state->garbage;  // (replicated deletes tag objects; only DB::delete enqueues garbage)
  cdb_apply_stats local;
  const cdb_status st = apply_ops_impl(ctx, state->k, state->nd, state->mb, *ops->b, pos, m->k, m->nd, m->mb,
                                       stats ? stats : &local);
  if (st != CDB_OK) return st;
  *out = m.release();
  return CDB_OK;
}

cdb_status cdb_encode_snapshot(cdb_ctx* ctx, cdb_merged* m, const cdb_encode_header* hdr, uint8_t** out,
                               size_t* len, cdb_encode_stats* stats) {
  if (!ctx || !m || !hdr || !out || !len) return CDB_BAD_ARGUMENT;
  if ((hdr->alias_len && !hdr->alias) || (hdr->addr_len && !hdr->addr) || (hdr->n_replicas && !hdr->replicas))
    return CDB_BAD_ARGUMENT;
  *out = nullptr;
  *len = 0;
  hipSetDevice(ctx->device);
  for (const auto& b : m->inputs)
    if (cdb_status st = refs_ready(ctx, b.get()); st != CDB_OK) return st;
  return encode_snapshot_impl(ctx, *m, *hdr, out, len, stats);
}

cdb_status cdb_encode_device(cdb_ctx* ctx, const cdb_dev_output* dout, cdb_batch* const* inputs, uint32_t n,
                             const cdb_encode_header* hdr, uint8_t** out, size_t* len, cdb_encode_stats* stats) {
  if (!ctx || !dout || !hdr || !out || !len || (n && !inputs)) return CDB_BAD_ARGUMENT;
  if ((hdr->alias_len && !hdr->alias) || (hdr->addr_len && !hdr->addr) || (hdr->n_replicas && !hdr->replicas))
    return CDB_BAD_ARGUMENT;
  if (n > 255) return fail(ctx, CDB_BAD_ARGUMENT, "at most 255 inputs behind one result");
  std::vector<Batch*> in(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (!inputs[i]) return CDB_BAD_ARGUMENT;
    in[i] = inputs[i]->b.get();
  }
  *out = nullptr;
  *len = 0;
  hipSetDevice(ctx->device);
  return encode_device_impl(ctx, *dout, in, *hdr, out, len, stats);
}

cdb_status cdb_crc64_gpu(cdb_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* crc) {
  if (!ctx || !crc || (len && !buf)) return CDB_BAD_ARGUMENT;
  hipSetDevice(ctx->device);
  return crc64_gpu_impl(ctx, buf, len, crc);
}

void cdb_merged_free(cdb_merged* m) { delete m; }
void cdb_free(void* p) { std::free(p); }

}  // extern "C"
