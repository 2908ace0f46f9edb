// omg_api.cpp — C-ABI (include/omg.h), device plan builder and the per-level
// orchestration of the FAS V-cycle / FMG on one GPU per rank.
//
// The control flow of every entry point follows the reference routine named in
// its comment (FermiQ/octree-mg, src/m_multigrid.f90 etc.); each per-box loop
// of the reference is one level-wide kernel launch here, and every MPI
// exchange of the reference (m_communication.f90:37-66) is one grouped RCCL
// send/recv round over xGMI carrying device-packed buffers.
#include <hip/hip_runtime.h>
#include <hipfft/hipfft.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <tuple>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/omg.h"
#include "omg_free.h"
#include "omg_free_gequad.h"
#include "omg_kernels.h"

using namespace omg;

namespace {

thread_local std::string g_last_error;

struct OmgError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                            \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess)                                                                    \
      throw OmgError(std::string(#x) + ": " + hipGetErrorString(e_) + " (" + __FILE__ + ":" + \
                     std::to_string(__LINE__) + ")");                                        \
  } while (0)

#define NCCLCHK(x)                                                                         \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) throw OmgError(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// Every place the host waits for a context stream goes through here, so the
// waits of a call can be counted (omg_host_sync_count: a multi-rank stand-alone
// V-cycle makes none unless max_res is requested).
inline void host_sync(omg_ctx* c, hipStream_t st) {
  c->n_host_syncs++;
  HIPCHK(hipStreamSynchronize(st));
}

template <typename F>
int guarded(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return 1;
  }
}

// Plan-only contexts (omg_ctx_create with OMG_DEVICE_NONE) build every host
// table of omg_tree_setup but allocate nothing on a device.
thread_local bool g_host_only = false;

template <typename T>
void dmalloc(T** p, size_t bytes, bool zero = false) {
  *p = nullptr;
  if (g_host_only || bytes == 0) return;
  HIPCHK(hipMalloc((void**)p, bytes));
  if (zero) HIPCHK(hipMemset(*p, 0, bytes));
}

template <typename T>
T* to_device(const std::vector<T>& v) {
  if (v.empty() || g_host_only) return nullptr;
  T* d = nullptr;
  HIPCHK(hipMalloc(&d, sizeof(T) * v.size()));
  HIPCHK(hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  return d;
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

const int kNeighbRev[6] = {2, 1, 4, 3, 6, 5};

// an on/off switch from the environment: set and not "0" (or empty)
bool env_flag(const char* name) {
  const char* v = getenv(name);
  return v && *v && std::strcmp(v, "0") != 0;
}

// a signalling NaN (quiet bit clear): OMG_DEBUG's poison
double snan_value() {
  const unsigned long long bits = 0x7FF4000000000000ULL;
  double d;
  std::memcpy(&d, &bits, 8);
  return d;
}

inline int pack_dix(const int d[3]) { return d[0] | (d[1] << 10) | (d[2] << 20); }

// ---------------------------------------------------------------------------
// tree helpers (reference src/m_data_structures.f90)
struct Tree {
  omg_ctx* c;
  int lvl(int id) const { return c->lvl[id - 1]; }
  int parent(int id) const { return c->parent[id - 1]; }
  int child(int id, int s) const { return c->children[(id - 1) * 8 + s - 1]; }
  int nbr(int id, int nb) const { return c->neighbors[(id - 1) * 6 + nb - 1]; }
  int rank(int id) const { return c->rank_of[id - 1]; }
  // mg_get_child_offset (m_data_structures.f90:456-467)
  void child_offset(int id, int d[3]) const {
    if (lvl(id) <= c->first_normal) {
      d[0] = d[1] = d[2] = 0;
    } else {
      for (int q = 0; q < 3; q++) d[q] = ((c->ix[(id - 1) * 3 + q] - 1) & 1) * (c->box_size >> 1);
    }
  }
};

// Level::d_topo, the per-box face words the tiled kernels load once
// (FaceTopo, omg_face.h), from the host tables; rebuilt when they change
// (phi_bc_store rewrites the physical faces' codes)
void pack_topo(Level& L) {
  if (!L.n) return;
  std::vector<int> w((size_t)L.n * 8, 0);
  auto put = [](int kind, long long arg) {
    if (arg < 0 || arg >= (1ll << 29)) throw OmgError("pack_topo: face argument out of range");
    return (int)(((unsigned)kind << 29) | (unsigned)arg);
  };
  for (int b = 0; b < L.n; b++) {
    unsigned nonlocal = 0;
    for (int f = 0; f < 6; f++) {
      const size_t i = (size_t)b * 6 + f;
      const int kind = L.h_nbk[i];
      long long arg = 0;
      if (kind == NB_LOCAL) {
        arg = L.h_nba[i];
      } else if (kind == NB_PHYS) {
        arg = -(long long)L.h_nba[i];
      } else if (kind == NB_REMOTE) {
        arg = L.h_sendpos[i];
      } else if (kind == NB_RB) {
        const RBRec& r = L.h_rb[L.h_nba[i]];
        if (r.coarse_idx < 0 || r.coarse_idx >= (1 << 25)) throw OmgError("pack_topo: coarse index out of range");
        arg = r.coarse_idx;
        for (int d = 0; d < 3; d++) {
          if (r.dix[d] != 0 && r.dix[d] != L.nc / 2) throw OmgError("pack_topo: child offset not 0 or nc/2");
          arg |= (long long)(r.dix[d] != 0) << (25 + d);
        }
      }
      if (kind != NB_LOCAL) nonlocal |= 1u << f;
      w[(size_t)b * 8 + f] = put(kind, arg);
    }
    w[(size_t)b * 8 + 6] = (int)nonlocal;
  }
  dfree(L.d_topo);
  L.d_topo = to_device(w);
}

Level* level_ptr(omg_ctx* c, int l) {
  auto it = c->levels.find(l);
  return it == c->levels.end() ? nullptr : &it->second;
}

LevelView empty_view() {
  LevelView v;
  std::memset(&v, 0, sizeof(v));
  return v;
}

LevelView view_of(omg_ctx* c, int l) {
  Level* L = level_ptr(c, l);
  return L ? L->view() : empty_view();
}

// Build a Transfer's device arrays from its per-peer lists.
void finalize_transfer(Transfer& T) {
  std::vector<int> s, r;
  int off = 0;
  for (auto& p : T.send) {
    p.offset = off;
    off += (int)p.items.size() / T.send_ints;
    s.insert(s.end(), p.items.begin(), p.items.end());
  }
  T.n_send = off;
  off = 0;
  for (auto& p : T.recv) {
    p.offset = off;
    off += (int)p.items.size() / T.recv_ints;
    r.insert(r.end(), p.items.begin(), p.items.end());
  }
  T.n_recv = off;
  T.d_send_items = to_device(s);
  T.d_recv_items = to_device(r);
}

// Group key-sorted (peer, key, item...) records into per-peer lists.
struct Rec {
  int peer;
  long long key;
  int a, b, c = 0;
};
std::vector<PeerList> group(std::vector<Rec>& recs, int ints_per_item) {
  std::sort(recs.begin(), recs.end(), [](const Rec& x, const Rec& y) {
    return x.peer != y.peer ? x.peer < y.peer : x.key < y.key;
  });
  std::vector<PeerList> out;
  for (auto& r : recs) {
    if (out.empty() || out.back().peer != r.peer) {
      out.push_back(PeerList());
      out.back().peer = r.peer;
    }
    out.back().keys.push_back(r.key);
    out.back().items.push_back(r.a);
    if (ints_per_item >= 2) out.back().items.push_back(r.b);
    if (ints_per_item >= 3) out.back().items.push_back(r.c);
  }
  return out;
}

}  // namespace

// ---------------------------------------------------------------------------
// In-process loopback transport.  n_ranks contexts of ONE process (one host
// thread each, typically sharing one GPU) exchange their transfer segments by
// device-to-device copies ordered with HIP events, instead of RCCL.  The plans,
// the packing/unpacking kernels, the wire order and the reductions are those
// of the RCCL path, so multi-rank parity can be checked on a single GPU.
struct omg_loop {
  struct Msg {
    const double* src;
    size_t n;
    hipEvent_t ev;
  };
  using Key = std::tuple<int, int, long long>;   // (from, to, sequence of that pair)
  int n_ranks = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::map<Key, Msg> box;
  std::map<Key, hipEvent_t> acks;               // (receiver, sender, seq) -> copies done
  std::map<long long, std::vector<double>> vals;
  std::map<long long, int> n_in, n_out;
};

// m_free_space's free_bc (src/m_free_space.f90:9-24) on the device: the FFT
// grid, the kernel spectrum, the boundary planes and the gather plan of the
// FFT level's right-hand side.
struct omg_free_state {
  bool initialized = false;
  int fft_lvl = INT_MIN;
  omg::FreeGrid G{};
  double r_min[3] = {0, 0, 0};       // mg%r_min of the domain
  double* d_R = nullptr;             // real padded grid [N3][N2][N1] (density, then potential)
  double2* d_Z = nullptr;            // its D2Z spectrum [N3][N2][N1/2+1]
  double* d_karray = nullptr;        // kernel spectrum * scal, same shape, real
  double* d_planes = nullptr;        // bc_x0, bc_x1, bc_y0, bc_y1, bc_z0, bc_z1
  hipfftHandle fwd = 0, inv = 0;
  bool have_plans = false;
  // my boxes at the FFT level: local index and ix
  int n_my = 0;
  int* d_my = nullptr;
  int* d_my_ix = nullptr;
  // the other ranks' boxes (multi-rank, FFT level not replicated)
  omg::Transfer gather;
  double* d_send = nullptr;
  double* d_recv = nullptr;
  int* d_recv_ix = nullptr;
  omg::FreePlaneGeom P{};
};

namespace {

constexpr char kLoopMagic[16] = "OMG-LOOPBACK-v1";
std::mutex g_loop_mu;
std::map<long long, std::shared_ptr<omg_loop>> g_loops;

template <typename Pred>
void loop_wait(omg_ctx* c, std::unique_lock<std::mutex>& lk, Pred pred, const std::string& what) {
  if (!c->loop->cv.wait_for(lk, std::chrono::seconds(60), pred))
    throw OmgError(std::string("loopback transport: rank ") + std::to_string(c->rank) +
                   " timed out waiting for " + what);
}

hipEvent_t loop_event(hipStream_t st) {
  hipEvent_t e;
  HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventRecord(e, st));
  return e;
}

void loop_exchange(omg_ctx* c, const Transfer& T, const double* sendbuf, double* recvbuf, hipStream_t st) {
  omg_loop& G = *c->loop;
  const size_t per = (size_t)T.item_doubles;
  const int me = c->rank;
  for (auto& p : T.send) {
    const size_t n = p.items.size() / T.send_ints * per;
    hipEvent_t ev = loop_event(st);
    std::lock_guard<std::mutex> lk(G.mu);
    G.box[{me, p.peer, c->loop_seq_send[p.peer]}] = {sendbuf + (size_t)p.offset * per, n, ev};
    G.cv.notify_all();
  }
  for (auto& p : T.recv) {
    const size_t n = p.items.size() / T.recv_ints * per;
    const omg_loop::Key k{p.peer, me, c->loop_seq_recv[p.peer]};
    omg_loop::Msg m;
    {
      std::unique_lock<std::mutex> lk(G.mu);
      loop_wait(c, lk, [&] { return G.box.count(k) > 0; },
                "a message from rank " + std::to_string(p.peer) + " (pair sequence " +
                    std::to_string(std::get<2>(k)) + ", " + std::to_string(n) + " doubles)");
      m = G.box[k];
      G.box.erase(k);
    }
    if (m.n != n) throw OmgError("loopback transport: message size mismatch");
    HIPCHK(hipStreamWaitEvent(st, m.ev, 0));
    HIPCHK(hipMemcpyAsync(recvbuf + (size_t)p.offset * per, m.src, n * sizeof(double),
                          hipMemcpyDeviceToDevice, st));
    HIPCHK(hipEventDestroy(m.ev));
  }
  for (auto& p : T.recv) {   // the sender may reuse its buffer once our copies ran
    hipEvent_t ev = loop_event(st);
    std::lock_guard<std::mutex> lk(G.mu);
    G.acks[{me, p.peer, c->loop_seq_recv[p.peer]++}] = ev;
    G.cv.notify_all();
  }
  for (auto& p : T.send) {
    const omg_loop::Key k{p.peer, me, c->loop_seq_send[p.peer]++};
    hipEvent_t ev;
    {
      std::unique_lock<std::mutex> lk(G.mu);
      loop_wait(c, lk, [&] { return G.acks.count(k) > 0; },
                "the acknowledgement of rank " + std::to_string(p.peer) + " (pair sequence " +
                    std::to_string(std::get<2>(k)) + ")");
      ev = G.acks[k];
      G.acks.erase(k);
    }
    HIPCHK(hipStreamWaitEvent(st, ev, 0));
    HIPCHK(hipEventDestroy(ev));
  }
}

// every rank's value, in rank order (the loopback MPI_Allgather)
std::vector<double> loop_allgather(omg_ctx* c, double v) {
  omg_loop& G = *c->loop;
  const long long s = c->loop_ar_seq++;
  std::unique_lock<std::mutex> lk(G.mu);
  auto& vals = G.vals[s];
  vals.resize(G.n_ranks);
  vals[c->rank] = v;
  G.n_in[s]++;
  G.cv.notify_all();
  loop_wait(c, lk, [&] { return G.n_in[s] == G.n_ranks; },
            "allreduce #" + std::to_string(s) + " (" + std::to_string(G.n_in[s]) + " ranks in)");
  std::vector<double> all = G.vals[s];
  if (++G.n_out[s] == G.n_ranks) {
    G.vals.erase(s);
    G.n_in.erase(s);
    G.n_out.erase(s);
  }
  return all;
}

// ---------------------------------------------------------------------------
// Host transport (omg_set_host_transport): the caller's messaging (the
// Fortran drop-in: MPI, the reference's own transport) over pinned host
// staging.  Every round waits on the host: the segments leave the device
// after the stream's work so far, arrive before anything queued after.
constexpr char kHostMagic[16] = "OMG-HOSTXPRT-v1";

double* host_stage(double*& p, size_t& cap, size_t n) {
  if (n > cap) {
    if (p) HIPCHK(hipHostFree(p));
    p = nullptr;
    HIPCHK(hipHostMalloc(&p, sizeof(double) * std::max<size_t>(n, 1)));
    cap = n;
  }
  return p;
}

void host_exchange(omg_ctx* c, const Transfer& T, const double* sendbuf, double* recvbuf, hipStream_t st) {
  if (!c->hx_exchange) throw OmgError("host transport: omg_set_host_transport was not called");
  const size_t per = (size_t)T.item_doubles;
  size_t ns = 0, nr = 0;
  for (auto& p : T.send) ns = std::max(ns, ((size_t)p.offset + p.items.size() / T.send_ints) * per);
  for (auto& p : T.recv) nr = std::max(nr, ((size_t)p.offset + p.items.size() / T.recv_ints) * per);
  double* hs = host_stage(c->h_xsend, c->h_xsend_n, ns);
  double* hr = host_stage(c->h_xrecv, c->h_xrecv_n, nr);
  std::vector<int> sp, rp;
  std::vector<long long> sn, rn;
  std::vector<const double*> sb;
  std::vector<double*> rb;
  for (auto& p : T.send) {
    const size_t n = p.items.size() / T.send_ints * per;
    HIPCHK(hipMemcpyAsync(hs + (size_t)p.offset * per, sendbuf + (size_t)p.offset * per, n * sizeof(double),
                          hipMemcpyDeviceToHost, st));
    sp.push_back(p.peer);
    sn.push_back((long long)n);
    sb.push_back(hs + (size_t)p.offset * per);
  }
  for (auto& p : T.recv) {
    rp.push_back(p.peer);
    rn.push_back((long long)(p.items.size() / T.recv_ints * per));
    rb.push_back(hr + (size_t)p.offset * per);
  }
  host_sync(c, st);
  if (c->hx_exchange(c->hx_user, (int)sp.size(), sp.data(), sn.data(), sb.data(), (int)rp.size(), rp.data(),
                     rn.data(), rb.data()) != 0)
    throw OmgError("host transport: the exchange callback failed");
  for (size_t i = 0; i < rp.size(); i++)
    HIPCHK(hipMemcpyAsync(recvbuf + (rb[i] - hr), rb[i], (size_t)rn[i] * sizeof(double), hipMemcpyHostToDevice,
                          st));
  host_sync(c, st);   // (the staging is reused by the next round)
}

std::vector<double> host_allgather(omg_ctx* c, double v) {
  if (!c->hx_allgather) throw OmgError("host transport: omg_set_host_transport was not called");
  std::vector<double> all(c->n_ranks);
  if (c->hx_allgather(c->hx_user, &v, 1, all.data()) != 0)
    throw OmgError("host transport: the allgather callback failed");
  return all;
}

// ---------------------------------------------------------------------------
// profiling: HIP events around kernel families on the context stream
constexpr int NO_LVL = INT_MIN;

// (on `st`, the context stream by default; with OMG_ROCTX set, a roctx range
// "name@lvl" around the host side of the step for rocprofv3 --marker-trace)
struct Prof {
  omg_ctx* c;
  const char* name;
  double cells;
  int lvl;
  hipStream_t st;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  bool range = false;
  Prof(omg_ctx* c_, const char* n, double cl, int l = NO_LVL, hipStream_t s = nullptr)
      : c(c_), name(n), cells(cl), lvl(l), st(s ? s : c_->stream) {
    if (c->roctx) {
      char buf[64];
      if (lvl == NO_LVL) std::snprintf(buf, sizeof(buf), "%s", name);
      else std::snprintf(buf, sizeof(buf), "%s@%d", name, lvl);
      roctxRangePushA(buf);
      range = true;
    }
    if (!c->profiling) return;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
  }
  ~Prof() {
    if (range) roctxRangePop();
    if (!e0) return;
    (void)hipEventRecord(e1, st);
    c->pending.push_back({name, e0, e1, cells, lvl});
  }
};

void resolve_stats(omg_ctx* c) {
  if (c->pending.empty()) return;
  for (auto& p : c->pending) {
    float ms = 0;
    HIPCHK(hipEventSynchronize(p.e1));
    HIPCHK(hipEventElapsedTime(&ms, p.e0, p.e1));
    for (int pass = 0; pass < (p.lvl == NO_LVL ? 1 : 2); pass++) {
      auto& s = c->stats[pass ? std::string(p.name) + "@" + std::to_string(p.lvl) : std::string(p.name)];
      s.launches++;
      s.ms += ms;
      s.cells += p.cells;
    }
    (void)hipEventDestroy(p.e0);
    (void)hipEventDestroy(p.e1);
  }
  c->pending.clear();
}

// One grouped RCCL round: send segment i to peer i, receive likewise
// (replaces sort_and_transfer_buffers, m_communication.f90:37-66).
void exchange(omg_ctx* c, const Transfer& T, const double* sendbuf, double* recvbuf, hipStream_t st = nullptr,
              int lvl = NO_LVL) {
  if (c->n_ranks == 1) return;
  if (T.send.empty() && T.recv.empty()) return;
  if (!st) st = c->stream;
  // "comm": one grouped round, timed on the stream it runs on; cells = the
  // doubles this rank receives
  Prof prof(c, st == c->stream ? "comm" : "comm_overlap", (double)T.n_recv * T.item_doubles, lvl, st);
  if (c->loop) {
    loop_exchange(c, T, sendbuf, recvbuf, st);
    return;
  }
  if (c->host_xport) {
    host_exchange(c, T, sendbuf, recvbuf, st);
    return;
  }
  ncclComm_t comm = (ncclComm_t)c->nccl;
  const size_t per = (size_t)T.item_doubles;
  NCCLCHK(ncclGroupStart());
  for (auto& p : T.send) {
    size_t n = p.items.size() / (T.send_ints) * per;
    NCCLCHK(ncclSend(sendbuf + (size_t)p.offset * per, n, ncclDouble, p.peer, comm, st));
  }
  for (auto& p : T.recv) {
    size_t n = p.items.size() / (T.recv_ints) * per;
    NCCLCHK(ncclRecv(recvbuf + (size_t)p.offset * per, n, ncclDouble, p.peer, comm, st));
  }
  NCCLCHK(ncclGroupEnd());
}

// ---------------------------------------------------------------------------
// Per-level steps
GcBC bc_for(omg_ctx* c, int lvl, int iv) {
  GcBC g;
  for (int nb = 0; nb < 6; nb++) {
    g.type[nb] = c->bc[iv - 1].type[nb];
    g.value[nb] = c->bc[iv - 1].value[nb];
  }
  auto it = c->d_face_off_lvl[iv - 1].find(lvl);
  g.face_off = it == c->d_face_off_lvl[iv - 1].end() ? nullptr : it->second;
  auto jt = c->d_face_type_lvl[iv - 1].find(lvl);
  g.face_type = jt == c->d_face_type_lvl[iv - 1].end() ? nullptr : jt->second;
  g.face_data = c->d_face_data[iv - 1];
  g.phi_stored = c->phi_bc_data_stored;
  return g;
}

// The refinement-boundary ghosts of level lvl+1 are interpolated from level
// lvl (its interior and tangential ghosts, box_gc_for_fine_neighbor,
// m_ghost_cells.f90:500-577): every write of phi on lvl makes them stale.
void rb_stale_above(omg_ctx* c, int lvl) {
  if (Level* U = level_ptr(c, lvl + 1)) {
    if (U->any_rb) U->phi_gc_ok = false;
    U->rbgv_ok = false;   // (its refinement-boundary coarse parts read lvl)
  }
}
// phi was written on a level: its ghost faces may no longer match a fill
void phi_dirty(omg_ctx* c, int lvl) {
  if (Level* L = level_ptr(c, lvl)) L->phi_gc_ok = L->gc_deferred = false;
  rb_stale_above(c, lvl);
}
void phi_dirty_all(omg_ctx* c) {
  for (auto& kv : c->levels) kv.second.phi_gc_ok = kv.second.rbgv_ok = kv.second.gc_deferred = false;
}

// Refinement-boundary faces whose ghosts a host callback sets instead of
// sides_rb (mg%bc(nb,iv)%refinement_bnd, fill_refinement_bnd,
// m_ghost_cells.f90:321-325): after a fill of the level has run on the device
// (sides_rb included), the coarse faces and the boxes go to the host, the
// callback sets the ghosts of face nb, and they come back.  Called once per
// fill, as the reference calls it once per fill.
void rb_host_fixup(omg_ctx* c, Level* L, int iv) {
  if (!c->rbh_any) return;
  auto it = L->rbh.find(iv);
  if (it == L->rbh.end() || it->second.n == 0) return;
  if (c->capturing) throw OmgError("refinement_bnd host callback inside a captured cycle");
  RbHostFaces& R = it->second;
  const int nc = L->nc, nc2 = nc * nc;
  const size_t per = (size_t)(nc + 2) * (nc + 2) * (nc + 2);
  launch_rbh_gather(L->view(), view_of(c, L->lvl - 1), iv, L->d_rb, R.d_items, R.d_slot, R.n, L->d_rbrecv, R.d_cgc,
                    R.d_cc, c->stream);
  HIPCHK(hipMemcpyAsync(R.h_cgc, R.d_cgc, sizeof(double) * R.n * nc2, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(R.h_cc, R.d_cc, sizeof(double) * R.n * per, hipMemcpyDeviceToHost, c->stream));
  host_sync(c, c->stream);
  for (int q0 = 0; q0 < R.n;) {   // one call per face direction (records sorted by face)
    int q1 = q0;
    while (q1 < R.n && R.nbs[q1] == R.nbs[q0]) q1++;
    const int nb = R.nbs[q0];
    auto fn = (omg_rb_fn)c->rb_fn[iv - 1][nb - 1];
    fn(c->rb_user[iv - 1][nb - 1], L->lvl, iv, q1 - q0, R.ids.data() + q0, R.nbs.data() + q0, nc,
       R.h_cgc + (size_t)q0 * nc2, R.h_cc + (size_t)q0 * per);
    q0 = q1;
  }
  HIPCHK(hipMemcpyAsync(R.d_cc, R.h_cc, sizeof(double) * R.n * per, hipMemcpyHostToDevice, c->stream));
  launch_rbh_scatter(L->view(), iv, R.d_items, R.n, R.d_cc, c->stream);
  host_sync(c, c->stream);   // (the pinned buffer is reused by the next fill)
}

void rbh_free(Level& L) {
  for (auto& kv : L.rbh) {
    RbHostFaces& R = kv.second;
    dfree(R.d_items);
    dfree(R.d_slot);
    dfree(R.d_cgc);
    dfree(R.d_cc);
    if (R.h_cgc) (void)hipHostFree(R.h_cgc);
    if (R.h_cc) (void)hipHostFree(R.h_cc);
  }
  L.rbh.clear();
}

// the records of every level with refinement boundaries, for the variables
// and faces that have a host callback
void rbh_build(omg_ctx* c) {
  c->rbh_any = false;
  for (int iv = 0; iv < kMaxVars; iv++)
    for (int nb = 0; nb < 6; nb++) c->rbh_any |= c->rb_fn[iv][nb] != nullptr;
  for (auto& kv : c->levels) {
    Level& L = kv.second;
    rbh_free(L);
    if (!c->rbh_any || !L.has_rb || !L.n || c->host_only) continue;
    // receive slot of every NB_RBREM face (its position in the rb exchange)
    std::map<int, int> rslot;
    {
      int pos = 0;
      for (auto& p : L.rbx.recv)
        for (int f : p.items) rslot[f] = pos++;
    }
    for (int iv = 1; iv <= c->n_vars; iv++) {
      RbHostFaces R;
      for (int nb = 1; nb <= 6; nb++) {
        if (!c->rb_fn[iv - 1][nb - 1]) continue;
        for (int b = 0; b < L.n; b++) {
          const int f = b * 6 + nb - 1, kind = L.h_nbk[f];
          if (kind != NB_RB && kind != NB_RBREM) continue;
          R.items.push_back(f);
          R.slot.push_back(kind == NB_RBREM ? rslot.at(f) : -1);
          R.ids.push_back(L.ids[b]);
          R.nbs.push_back(nb);
        }
      }
      R.n = (int)R.items.size();
      if (!R.n) continue;
      const size_t nc2 = (size_t)L.nc * L.nc, per = (size_t)(L.nc + 2) * (L.nc + 2) * (L.nc + 2);
      R.d_items = to_device(R.items);
      R.d_slot = to_device(R.slot);
      dmalloc(&R.d_cgc, sizeof(double) * R.n * nc2);
      dmalloc(&R.d_cc, sizeof(double) * R.n * per);
      HIPCHK(hipHostMalloc(&R.h_cgc, sizeof(double) * R.n * nc2));
      HIPCHK(hipHostMalloc(&R.h_cc, sizeof(double) * R.n * per));
      L.rbh[iv] = std::move(R);
    }
  }
}

// halo exchange of the faces packed by the last fill/substep kernel, then
// fill_buffered_nb (m_ghost_cells.f90:163-174, 424-454); rb_hook: the fill is
// complete here (no full fill follows), so host refinement-boundary callbacks run
void finish_rb(omg_ctx* c, Level* L, int iv);
void finish_halo(omg_ctx* c, Level* L, int iv, bool rb_hook = true) {
  if (c->n_ranks > 1) {
    if (L->halo.n_send || L->halo.n_recv) {
      exchange(c, L->halo, L->d_sendbuf, L->d_recvbuf, nullptr, L->lvl);
      launch_unpack_faces(L->view(), iv, L->halo.d_recv_items, L->halo.n_recv, L->d_recvbuf, c->stream);
    }
    finish_rb(c, L, iv);
  }
  if (rb_hook) rb_host_fixup(c, L, iv);
}

// refinement boundaries across ranks (buffer_refinement_boundaries,
// m_ghost_cells.f90:157-162, 200-229): coarse faces go out interpolated,
// the fine side applies sides_rb once they arrive
void finish_rb(omg_ctx* c, Level* L, int iv) {
  if (c->n_ranks == 1) return;
  if (L->rbx.n_send || L->rbx.n_recv) {
    launch_rb_pack(view_of(c, L->lvl - 1), iv, L->rbx.d_send_items, L->rbx.n_send, L->nc, L->d_rbsend,
                   c->stream);
    exchange(c, L->rbx, L->d_rbsend, L->d_rbrecv, nullptr, L->lvl);
    launch_rb_unpack(L->view(), iv, L->rbx.d_recv_items, L->rbx.n_recv, L->d_rbrecv, c->stream);
  }
}

// mg_fill_ghost_cells_lvl (m_ghost_cells.f90:131-175): same-GPU faces are
// pushed by their owner, physical / refinement-boundary ghosts recomputed,
// remote faces packed, exchanged over RCCL and unpacked.
void fill_gc_lvl(omg_ctx* c, int lvl, int iv) {
  if (lvl < c->lowest) throw OmgError("fill_ghost_cells_lvl: lvl < lowest_lvl");
  if (lvl > c->highest) throw OmgError("fill_ghost_cells_lvl: lvl > highest_lvl");
  Level* L = level_ptr(c, lvl);
  if (!L) return;
  if (iv == 1) {
    L->phi_gc_ok = true;
    L->gc_deferred = false;
    rb_stale_above(c, lvl);   // (the ghosts it sets are read by lvl+1's interpolation)
  }
  if (L->n) {
    Prof p(c, "fill_gc", (double)L->n * 6 * L->nc * L->nc, lvl);
    if (iv != 1 || L->has_rb || c->no_fill_tile ||
        !launch_fill_tile(L->sweep_view(), bc_for(c, lvl, iv), L->d_sendbuf, c->stream))
      launch_fill_gc(L->view(), iv, 3, view_of(c, lvl - 1), L->d_rb, bc_for(c, lvl, iv), L->d_sendbuf,
                     c->stream);
  }
  finish_halo(c, L, iv);
}

// Deep halo of a split level (plan_deep) around a k_gsrb3 / k_gsrb4 pass:
// before it, the proxies get phi of the colour the pass reads (as stored: a
// pending mean shift is subtracted by the pass from proxies and own boxes
// alike) and, when the level's rhs changed since the last fill, rhs; after
// it, the ghosts of this rank's faces toward other GPUs (nobody pushed them)
// by the level's halo plan.  Both rounds are collective: the rhs refill is
// decided by flags every rank changes alike (every rhs writer is a
// collective call, include/omg.h), checked under OMG_CHECK_COLLECTIVE.
double allreduce(omg_ctx* c, double v, bool is_max);
void deep_before(omg_ctx* c, Level* L, int colour) {
  if (!L->deep) return;
  const LevelView V = L->view();
  if (c->check_collective && (allreduce(c, L->prox_rhs_ok ? 1.0 : 0.0, true) > 0.5) != L->prox_rhs_ok)
    throw OmgError("deep halo: the rhs refill decision differs across ranks (an rhs write was not collective)");
  if (!L->prox_rhs_ok) {
    Prof p(c, "deep_rhs", (double)L->deep_rhs.n_recv * 64, L->lvl);
    launch_deep_copy(V, 2, 0, 64, L->deep_rhs.d_send_items, L->deep_rhs.n_send, L->d_sendbuf, false, c->stream);
    exchange(c, L->deep_rhs, L->d_sendbuf, L->d_recvbuf, nullptr, L->lvl);
    launch_deep_copy(V, 2, 0, 64, L->deep_rhs.d_recv_items, L->deep_rhs.n_recv, L->d_recvbuf, true, c->stream);
    L->prox_rhs_ok = true;
  }
  Prof p(c, "deep_phi", (double)L->deep_phi.n_recv * 32, L->lvl);
  launch_deep_copy(V, 1, colour, 32, L->deep_phi.d_send_items, L->deep_phi.n_send, L->d_sendbuf, false, c->stream);
  exchange(c, L->deep_phi, L->d_sendbuf, L->d_recvbuf, nullptr, L->lvl);
  launch_deep_copy(V, 1, colour, 32, L->deep_phi.d_recv_items, L->deep_phi.n_recv, L->d_recvbuf, true, c->stream);
}
// defer: on the comm stream, joined by the caller (faces_pending: only the
// boxes with a face on another GPU wait for it, update_coarse's residual)
void deep_after(omg_ctx* c, Level* L, bool defer = false) {
  if (!L->deep) return;
  hipStream_t st = c->stream;
  if (defer && L->n_bnd && L->n_int) {
    HIPCHK(hipEventRecord(c->ev_bnd, c->stream));
    HIPCHK(hipStreamWaitEvent(c->stream_comm, c->ev_bnd, 0));
    st = c->stream_comm;
    L->faces_pending = true;
  }
  Prof p(c, "deep_faces", (double)L->halo.n_recv * L->nc * L->nc, L->lvl, st);
  launch_face_pack(L->view(), 1, L->halo.d_send_items, L->halo.n_send, L->d_sendbuf, st);
  exchange(c, L->halo, L->d_sendbuf, L->d_recvbuf, st, L->lvl);
  launch_unpack_faces(L->view(), 1, L->halo.d_recv_items, L->halo.n_recv, L->d_recvbuf, st);
  if (L->faces_pending) HIPCHK(hipEventRecord(c->ev_comm, c->stream_comm));
}
// after a deep level's RES pass (res = phi - old, stored for the correction
// form above): the proxies get res where the level above's columns read it
// (the bricks of the deep halo, both colours), and this rank's faces toward
// other GPUs get their res ghosts (the halo plan), as the pass gave the
// same-GPU ones
void deep_res(omg_ctx* c, Level* L) {
  if (!L->deep) return;
  const LevelView V = L->view();
  Prof p(c, "deep_res", (double)L->deep_rhs.n_recv * 64, L->lvl);
  launch_deep_copy(V, 4, 0, 64, L->deep_rhs.d_send_items, L->deep_rhs.n_send, L->d_sendbuf, false, c->stream);
  exchange(c, L->deep_rhs, L->d_sendbuf, L->d_recvbuf, nullptr, L->lvl);
  launch_deep_copy(V, 4, 0, 64, L->deep_rhs.d_recv_items, L->deep_rhs.n_recv, L->d_recvbuf, true, c->stream);
  launch_face_pack(V, 4, L->halo.d_send_items, L->halo.n_send, L->d_sendbuf, c->stream);
  exchange(c, L->halo, L->d_sendbuf, L->d_recvbuf, nullptr, L->lvl);
  launch_unpack_faces(V, 4, L->halo.d_recv_items, L->halo.n_recv, L->d_recvbuf, c->stream);
}

// the deferred faces of deep_after have arrived (the main stream waits)
void faces_join(omg_ctx* c, Level* L) {
  if (!L || !L->faces_pending) return;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_comm, 0));
  L->faces_pending = false;
}

void materialize_level(omg_ctx* c, Level* L);
void drop_rhs_lex(omg_ctx* c);
void phi_mean_ready(omg_ctx* c);
double* red_mean(omg_ctx* c, int ch);

// smooth_boxes (m_multigrid.f90:404-424)
// want_res: the level above takes k_gsrb3's correct_children form next, which
// reads this level's res = phi - old: the last three substeps run as one
// k_gsrb3 pass that also stores it (the plain substeps first); returns whether
// that pass ran.
// four: runs of four substeps as one k_gsrb4 pass (the down-smoothing when
// the residual + restriction run unfused after it, OMG_BLOCK4)
// defer_faces: a k_gsrb4 pass that ends the smoothing leaves its remote faces'
// exchange in flight on the comm stream (deep_after), for update_coarse
bool b3_usable(omg_ctx* c, int lvl, B3Phys& P, const B3Phys*& ph);
bool smooth_boxes(omg_ctx* c, int lvl, int n_cycle, int first_substep = 1, int skip_last = 0,
                  bool want_res = false, bool four = false, bool defer_faces = false) {
  Level* L = level_ptr(c, lvl);
  const int n_sub = n_cycle * c->n_substeps - skip_last;
  bool res_done = false;
  if (!L) return false;
  if (n_sub >= 1) rb_stale_above(c, lvl);
  // a pending phi shift is subtracted by the first tiled substep while it
  // loads (the values it reads are dead afterwards); otherwise applied now
  // (not next to refinement boundaries: their ghosts read the coarse level;
  // nor before a block pass with physical faces, whose ghosts take no shift)
  const bool absorb = L->shift_pending && c->smoother == OMG_SMOOTHER_GSRB && n_sub >= 1 &&
                      (L->phi_gc_ok || L->gc_deferred) &&
                      !L->has_rb && gs_tiled(L->nc, c->op, L->has_rb) && !(L->d_b3 && L->b3_phys);
  if (L->shift_pending && !absorb) materialize_level(c, L);
  if (c->smoother != OMG_SMOOTHER_GSRB) {
    // the register-ring kernel reads rhs from its ring-order copy, rebuilt
    // here when a write since the last build dropped it (update_coarse for
    // the levels below the top, every entry point that may change rhs)
    const bool ring = n_sub >= 1 && L->d_rhs_lex && gs_lex_ring_ok(L->nc, c->op);
    if (ring && !L->rhs_lex_ok) {
      Prof p(c, "rhs_lex", (double)L->n * L->nc * L->nc * L->nc, lvl);
      launch_rhs_lex(L->view(), L->d_rhs_lex, c->stream);
      L->rhs_lex_ok = true;
    }
    // the register ring also writes the boxes' new x boundary layers, so the
    // fill after each sweep stages 12 KB per box instead of 32 (no
    // refinement boundaries on the level; OMG_NO_FILL_XL: the plain fill)
    const bool xlf = ring && L->d_xlay && !L->has_rb && !c->no_fill_tile && !c->no_fill_xl;
    // Round 4: an even number of ring sweeps on a level whose faces are
    // same-GPU or physical runs with no fill in between: sweep n reads the
    // ghost set sweep n-1 pushed into (the box storage's own faces for odd
    // n, d_galt for even n; every sweep after the first forms the physical
    // ghosts at load, since only the same-GPU faces are pushed), so the last
    // sweep lands in the box storage and only its physical ghosts are left to
    // form (k_phys_gc).  The reference fills after every sweep
    // (m_multigrid.f90:412-423): the same values reach the same ghosts
    // before every read.  OMG_NO_GS_DBL: the fill after every sweep.
    // (d_galt exists only where no fill of this level exchanges anything:
    // no remote faces, no refinement-boundary faces, and no coarse faces
    // this rank owes another rank's refinement boundaries, ensure_rhs_lex.)
    if (xlf && L->d_galt && n_sub % 2 == 0 && L->n && !c->no_gs_dbl) {
      const GcBC bc = bc_for(c, lvl, 1);
      double* prim = L->d_phi + 2 * (long long)L->view().hv;
      for (int n = 1; n <= n_sub; n++) {
        const bool odd = n & 1;
        GhostSets gs;
        gs.in = odd ? prim : L->d_galt;
        gs.in_stride = odd ? L->stride : 6 * (long long)stored_face(L->nc);
        gs.out = odd ? L->d_galt : prim;
        gs.out_stride = odd ? 6 * (long long)stored_face(L->nc) : L->stride;
        gs.phys_load = n > 1;
        Prof p(c, "smoother_gs", (double)L->n * L->nc * L->nc * L->nc, lvl);
        launch_gs_lex(L->view(), c->op, c->lambda, c->stream, L->d_rhs_lex, nullptr, &gs, &bc);
      }
      if (L->n_physbox) {
        Prof p(c, "fill_gc", (double)L->n_physbox * 6 * L->nc * L->nc, lvl);
        launch_phys_gc(L->view(), bc, L->d_physbox, L->n_physbox, c->stream);
      }
      L->phi_gc_ok = true;
      return false;
    }
    for (int n = 1; n <= n_sub; n++) {
      if (L->n) {
        Prof p(c, "smoother_gs", (double)L->n * L->nc * L->nc * L->nc, lvl);
        launch_gs_lex(L->view(), c->op, c->lambda, c->stream, ring ? L->d_rhs_lex : nullptr,
                      xlf ? L->d_xlay : nullptr);
      }
      if (xlf) {
        L->phi_gc_ok = true;
        if (L->n) {
          Prof p(c, "fill_gc", (double)L->n * 6 * L->nc * L->nc, lvl);
          launch_fill_tile_xl(L->sweep_view(), bc_for(c, lvl, 1), L->d_sendbuf, L->d_xlay, c->stream);
        }
        finish_halo(c, L, 1);
      } else {
        fill_gc_lvl(c, lvl, 1);
      }
    }
    return false;
  }
  for (int n = first_substep; n <= n_sub; n++) {
    // substep n updates the cells with i+j+k+n even, i.e. colour e = n mod 2,
    // and ends with the ghost fill; same-GPU neighbours only need colour e
    // when their ghost faces were consistent before the substep.
    // For odd box sizes the box-local colouring is not global (a ghost has the
    // colour of the cell it is read by), so nothing is pushed during the
    // substep and a full fill follows it.
    const int e = n & 1;
    const bool odd = L->nc & 1;
    if (n == 1 && absorb) phi_mean_ready(c);
    const double* shift = (n == 1 && absorb) ? red_mean(c, 0) : nullptr;
    if (n == 1) L->shift_pending = false;
    // substeps n, n+1, n+2 in one pass (k_gsrb3) into phi's other buffer: it
    // reads the neighbours' cells in their boxes, which equal its ghosts only
    // when they are consistent (phi_gc_ok), and writes every ghost face
    // (ph: the ghosts across physical faces, formed in the pass)
    B3Phys P3;
    const B3Phys* ph = nullptr;
    const bool b3 = b3_usable(c, lvl, P3, ph);
    if (four && (n_sub - n + 1) % 4 == 0 && b3 && (!ph || c->block4_phys)) {
      double* other = L->d_phi == L->d_data ? L->d_phi_buf : L->d_data;
      deep_before(c, L, 1 - e);
      {
        Prof p(c, "smoother_gsrb4", 2.0 * L->n * L->nc * L->nc * L->nc, lvl);
        launch_gsrb4(L->view(), other, L->d_b3, L->n_b3, c->op, c->lambda, e, shift, c->stream, nullptr, nullptr,
                     ph);
      }
      L->d_phi = other;
      if (L->gc_deferred) L->phi_gc_ok = true, L->gc_deferred = false;   // (it wrote every ghost face)
      deep_after(c, L, defer_faces && n + 3 == n_sub);
      n += 3;
      continue;
    }
    if (n + 2 <= n_sub && b3 && !(want_res && (n_sub - n + 1) % 3 != 0)) {
      double* other = L->d_phi == L->d_data ? L->d_phi_buf : L->d_data;
      // the down-smoothing's last pass before k_smooth_resid (skip_last: it
      // runs the next substep, colour 0, and forms colour 0's ghosts itself
      // from colour 1, reading colour 1's only): push colour e = 1 alone
      // (a split level: both colours, its remote faces' ghosts arrive whole)
      const bool push1 = L->deep || !(skip_last == 1 && n + 2 == n_sub && e == 1);
      const bool res = want_res && n + 2 == n_sub && push1;
      deep_before(c, L, 1 - e);
      {
        Prof p(c, res ? "smoother_gsrb3r" : "smoother_gsrb3", 1.5 * L->n * L->nc * L->nc * L->nc, lvl);
        launch_gsrb3(L->view(), other, L->d_b3, L->n_b3, c->op, c->lambda, e, shift, c->stream, push1, nullptr,
                     nullptr, 1, res, ph);
      }
      res_done = res;
      L->d_phi = other;
      // (its ghost faces: every one, colour e's only without push1, whose
      // colour-(1-e) halves k_smooth_resid forms itself)
      if (L->gc_deferred) L->phi_gc_ok = true, L->gc_deferred = false;
      deep_after(c, L);
      if (res) deep_res(c, L);
      n += 2;
      continue;
    }
    // (the one-substep kernels read the ghosts: a deferred fill runs first)
    if (L->gc_deferred) fill_gc_lvl(c, lvl, 1);
    if (L->n_bnd && L->n_int && !odd && gs_tiled(L->nc, c->op, L->has_rb)) {
      // boxes with faces on other GPUs first; their halo travels on the comm
      // stream while the interior boxes run (the substep reads only its own
      // box's ghost faces, and an interior box has no remote one; the unpack
      // writes remote faces only)
      const int gvm = L->d_rbgv ? (L->rbgv_ok ? 2 : 1) : 0;
      if (gvm) L->rbgv_ok = true;
      {
        Prof p(c, "smoother_gsrb", 0.5 * L->n_bnd * L->nc * L->nc * L->nc, lvl);
        launch_gs_substep(L->sweep_view(), c->op, c->lambda, e, 1 << e, view_of(c, lvl - 1), L->d_rb, L->has_rb,
                          bc_for(c, lvl, 1), L->d_sendbuf, shift, c->stream, L->d_bnd, L->n_bnd, L->d_rbgv, gvm);
      }
      HIPCHK(hipEventRecord(c->ev_bnd, c->stream));
      // the interior boxes are queued before the exchange is issued: the
      // exchange may wait on the host (the loopback transport waits for its
      // peer's message), and the interior substep needs nothing from it
      {
        Prof p(c, "smoother_gsrb", 0.5 * L->n_int * L->nc * L->nc * L->nc, lvl);
        launch_gs_substep(L->sweep_view(), c->op, c->lambda, e, 1 << e, view_of(c, lvl - 1), L->d_rb, L->has_rb,
                          bc_for(c, lvl, 1), L->d_sendbuf, shift, c->stream, L->d_int, L->n_int, L->d_rbgv, gvm);
      }
      HIPCHK(hipStreamWaitEvent(c->stream_comm, c->ev_bnd, 0));
      exchange(c, L->halo, L->d_sendbuf, L->d_recvbuf, c->stream_comm, lvl);
      launch_unpack_faces(L->view(), 1, L->halo.d_recv_items, L->halo.n_recv, L->d_recvbuf, c->stream_comm);
      HIPCHK(hipEventRecord(c->ev_comm, c->stream_comm));
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_comm, 0));
      finish_rb(c, L, 1);
      if (!L->phi_gc_ok) fill_gc_lvl(c, lvl, 1);
      else rb_host_fixup(c, L, 1);
      continue;
    }
    if (L->n) {
      Prof p(c, "smoother_gsrb", 0.5 * L->n * L->nc * L->nc * L->nc, lvl);
      // refinement-boundary coarse parts: the first substep after the level
      // below changed computes and stores them, the others read them
      const int gvm = L->d_rbgv ? (L->rbgv_ok ? 2 : 1) : 0;
      if (gvm) L->rbgv_ok = true;
      launch_gs_substep(L->sweep_view(), c->op, c->lambda, e, odd ? 0 : 1 << e, view_of(c, lvl - 1), L->d_rb,
                        L->has_rb, bc_for(c, lvl, 1), L->d_sendbuf, shift, c->stream, nullptr, 0, L->d_rbgv, gvm);
    }
    const bool full_fill = odd || !L->phi_gc_ok;
    finish_halo(c, L, 1, !full_fill);
    if (full_fill) fill_gc_lvl(c, lvl, 1);
  }
  return res_done;
}

bool tiled_level(omg_ctx* c, const Level* L) {
  (void)c;
  return L && tiled_nc(L->nc);
}

void residual_lvl(omg_ctx* c, int lvl, unsigned long long* maxbits) {
  Level* L = level_ptr(c, lvl);
  if (!L || L->n == 0) return;
  Prof p(c, "residual", (double)L->n * L->nc * L->nc * L->nc, lvl);
  if (tiled_level(c, L))
    launch_resid_restrict(L->sweep_view(), empty_view(), c->op, c->lambda, maxbits, 0, nullptr, nullptr, c->stream);
  else
    launch_residual(L->view(), c->op, c->lambda, maxbits, c->stream);
}

// max over levels lo..hi of max_residual_lvl (m_multigrid.f90:296-311), this
// rank only: the levels' maxima fold into one word on the device, read back
// with one synchronisation
double max_residual_levels(omg_ctx* c, int lo, int hi) {
  unsigned long long* d = (unsigned long long*)c->d_scalar;
  for (int l = lo; l <= hi; l++) {
    residual_lvl(c, l, c->d_maxslots);
    launch_max_fold(c->d_maxslots, d, l > lo, c->stream);
  }
  HIPCHK(hipMemcpyAsync(c->h_scalar, d, 8, hipMemcpyDeviceToHost, c->stream));
  if (c->capturing) {   // run_cycle reads it once the graph has run
    if (c->max_deferred) throw OmgError("internal: two max-residual readbacks in one captured cycle");
    c->max_deferred = true;
    return 0.0;
  }
  host_sync(c, c->stream);
  return c->h_scalar[0];
}

double max_residual_lvl(omg_ctx* c, int lvl) { return max_residual_levels(c, lvl, lvl); }

// the remote part of mg_restrict_lvl: children whose parent lives on another
// rank are restricted into a buffer, exchanged and unpacked (m_restrict.f90:
// 94-108, 196-211)
void restrict_remote(omg_ctx* c, int iv, int lvl) {
  Level* F = level_ptr(c, lvl);
  Level* C = level_ptr(c, lvl - 1);
  if (c->n_ranks > 1 && F && C && (F->restr.n_send || F->restr.n_recv)) {
    launch_restrict_pack(F->view(), iv, F->restr.d_send_items, F->restr.n_send, F->d_sendbuf, c->stream);
    exchange(c, F->restr, F->d_sendbuf, C->d_recvbuf, nullptr, lvl);
    launch_restrict_unpack(C->view(), iv, F->restr.d_recv_items, F->restr.n_recv, F->nc / 2, C->d_recvbuf,
                           c->stream);
  }
}

// mg_restrict_lvl (m_restrict.f90:83-114)
void restrict_lvl(omg_ctx* c, int iv, int lvl) {
  if (lvl <= c->lowest) throw OmgError("cannot restrict lvl <= lowest_lvl");
  if (iv == 1) phi_dirty(c, lvl - 1);
  Level* F = level_ptr(c, lvl);
  restrict_remote(c, iv, lvl);
  if (F && F->n_pairs) {
    Prof p(c, "restrict", (double)F->n_pairs * F->nc * F->nc * F->nc, lvl);
    launch_restrict(F->view(), view_of(c, lvl - 1), iv, F->d_pairs, F->n_pairs, F->d_parent_local, F->d_dix,
                    c->stream);
  }
}

// mg_prolong (m_prolong.f90:51-85), lvl -> lvl+1
void prolong(omg_ctx* c, int lvl, int iv, int iv_to, int add) {
  if (lvl == c->highest) throw OmgError("cannot prolong highest level");
  if (lvl < c->lowest) throw OmgError("cannot prolong below lowest level");
  if (iv_to == 1) phi_dirty(c, lvl + 1);
  Level* F = level_ptr(c, lvl + 1);
  Level* C = level_ptr(c, lvl);
  const LevelView FV = view_of(c, lvl + 1), CV = view_of(c, lvl);
  if (c->n_ranks > 1 && F && C && (F->prol.n_send || F->prol.n_recv)) {
    launch_prolong_pack(CV, FV, iv, F->prol.d_send_items, F->prol.n_send, C->d_sendbuf, c->stream);
    exchange(c, F->prol, C->d_sendbuf, F->d_recvbuf, nullptr, lvl + 1);
    launch_prolong_unpack(FV, iv_to, add, F->prol.d_recv_items, F->prol.n_recv, F->d_recvbuf,
                          c->stream);
  }
  if (F && F->n_pairs) {
    Prof p(c, "prolong", (double)F->n_pairs * F->nc * F->nc * F->nc, lvl + 1);
    launch_prolong(CV, FV, iv, iv_to, add, F->d_pairs, F->n_pairs, F->d_parent_local, F->d_dix,
                   c->stream);
  }
}

// Whether the down-smoothing of level lvl can end in k_smooth_resid (its last
// substep, colour 0, fused with update_coarse's residual + restriction):
// red-black (two substeps per cycle, so the last one is colour 0),
// Laplacian / Helmholtz, 16^3 or 8^3 boxes.  Same-GPU faces: the recomputed
// ghosts read the neighbour box directly; physical and refinement-boundary
// faces (round 4; OMG_NO_FUSE_DOWN_BC: not fused): from the box's own cells.
// On a level with faces on other GPUs only the boxes without such a face fuse
// (n_int > 0); the others take the unfused substep + residual.
bool smooth_resid_ok(omg_ctx* c, int lvl) {
  const Level* F = level_ptr(c, lvl);
  const Level* C = level_ptr(c, lvl - 1);
  // (a host refinement_bnd callback sets phi's ghosts on some faces: the
  // kernel's sides_rb would stand in for it)
  if (F) {
    const auto rbh = F->rbh.find(1);
    if (rbh != F->rbh.end() && rbh->second.n) return false;
  }
  return !c->no_fuse_down && F && C && F->n && c->smoother == OMG_SMOOTHER_GSRB && c->n_substeps == 2 &&
         c->n_cycle_down >= 1 &&
         (c->op == OP_LPL || c->op == OP_HELM) && (F->nc == 16 || F->nc == 8) &&
         !(c->no_fuse_down_bc && (F->has_rb || F->has_phys)) && (!F->has_remote || F->n_int) &&
         // Refinement-boundary faces whose coarse box is on another rank
         // exchange coarse faces after every substep (finish_rb); the fused
         // kernel forms those ghosts from the coarse box itself.  Decided
         // alike on every rank (any_rbx: the global tree).  Physical and
         // same-GPU refinement-boundary faces fuse on split levels too
         // (update_coarse: the boundary boxes' substep leaves the colour-1
         // halves of those ghosts for the fused boxes' edge taps).
         !F->any_rbx;
}

// update_coarse (m_multigrid.f90:347-384); fused: the level's last down
// substep is still to do (smooth_resid_ok), k_smooth_resid runs it
// with tail_crhs the coarse tail forms lvl-1's ghosts and coarse rhs itself
// (its top level, TailArgs::top_crhs): only the residual and the restriction here
void update_coarse(omg_ctx* c, int lvl, bool fused = false, bool tail_crhs = false) {
  Level* F = level_ptr(c, lvl);
  if (Level* Cl = level_ptr(c, lvl - 1)) {
    Cl->rhs_lex_ok = Cl->prox_rhs_ok = false;   // its rhs is rewritten below
    // restriction overwrites every box of an all-parents level (interior), and
    // the fill below every ghost face: a pending shift there is dead
    if (Cl->all_parents) Cl->shift_pending = false;
    else materialize_level(c, Cl);
  }
  if (F && F->n && tiled_level(c, F)) {
    // The stored refinement-boundary coarse parts of lvl (d_rbgv) were formed
    // from lvl-1 as it stands until the restriction below writes it, which is
    // what the fused down-substep's ghosts need; read the flag before
    // phi_dirty drops it.  (The coarse boxes across those faces are leaves:
    // the restriction never writes them.)
    const bool rbgv = F->rbgv_ok;
    // residual + restriction of phi and res in one pass (omg_tiles.hip)
    phi_dirty(c, lvl - 1);
    if (fused && F->has_remote) {
      // multi-GPU: boxes with a face on another GPU take the unfused pair (the
      // substep, its halo on the comm stream, then the residual); the others
      // run fused meanwhile.  Those read their neighbours' colour-1 ghosts at
      // face edges, and some of those faces are remote: the unpack therefore
      // writes the colour-0 halves only (the colour this substep changed;
      // colour 1 is consistent since the previous substep's exchange).
      // Physical and refinement-boundary ghosts: a fused box's edge tap reads
      // its neighbour's colour-1 ghost on the neighbour's side face as it
      // stood before this substep, so the boundary boxes' substep writes only
      // the colour-0 halves of those ghosts (colours bit 2), and k_face_gc
      // forms them whole once the fused launch is done, before the boundary
      // boxes' residual reads them.
      const bool faces = F->any_phys || F->any_rb;
      {
        Prof p(c, "smoother_gsrb", 0.5 * F->n_bnd * F->nc * F->nc * F->nc, lvl);
        launch_gs_substep(F->view(), c->op, c->lambda, 0, faces ? 1 | 4 : 1, view_of(c, lvl - 1), F->d_rb,
                          F->has_rb, bc_for(c, lvl, 1), F->d_sendbuf, nullptr, c->stream, F->d_bnd, F->n_bnd,
                          rbgv ? F->d_rbgv : nullptr, rbgv ? 2 : 0);
      }
      HIPCHK(hipEventRecord(c->ev_bnd, c->stream));
      {   // (queued before the exchange is issued, as in smooth_boxes)
        Prof p(c, "smooth_resid", (double)F->n_int * F->nc * F->nc * F->nc, lvl);
        if (!launch_smooth_resid(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, 1, F->d_parent_local,
                                 F->d_dix, c->stream, F->d_int, F->n_int, bc_for(c, lvl, 1), F->has_rb, F->has_phys,
                                 rbgv ? F->d_rbgv : nullptr))
          throw OmgError("smooth_resid: not available for this level");
      }
      HIPCHK(hipStreamWaitEvent(c->stream_comm, c->ev_bnd, 0));
      exchange(c, F->halo, F->d_sendbuf, F->d_recvbuf, c->stream_comm, lvl);
      launch_unpack_faces(F->view(), 1, F->halo.d_recv_items, F->halo.n_recv, F->d_recvbuf, c->stream_comm, 1);
      HIPCHK(hipEventRecord(c->ev_comm, c->stream_comm));
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_comm, 0));
      if (faces && F->n_bndface) {
        Prof p(c, "face_gc", (double)F->n_bndface * 6 * F->nc * F->nc, lvl);
        launch_face_gc(F->view(), view_of(c, lvl - 1), bc_for(c, lvl, 1), F->d_bndface, F->n_bndface, c->stream);
      }
      {
        Prof p(c, "resid_restrict", (double)F->n_bnd * F->nc * F->nc * F->nc, lvl);
        launch_resid_restrict(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, nullptr, 1, F->d_parent_local,
                              F->d_dix, c->stream, F->d_bnd, F->n_bnd);
      }
    } else if (fused) {
      Prof p(c, "smooth_resid", (double)F->n * F->nc * F->nc * F->nc, lvl);
      if (!launch_smooth_resid(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, 1, F->d_parent_local,
                               F->d_dix, c->stream, nullptr, 0, bc_for(c, lvl, 1), F->has_rb, F->has_phys,
                               rbgv ? F->d_rbgv : nullptr))
        throw OmgError("smooth_resid: not available for this level");
    } else if (F->faces_pending) {
      // a split level's k_gsrb4 pass left its remote faces' ghosts in flight
      // (deep_after): the boxes without such a face first
      {
        Prof p(c, "resid_restrict", (double)F->n_int * F->nc * F->nc * F->nc, lvl);
        launch_resid_restrict(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, nullptr, 1, F->d_parent_local,
                              F->d_dix, c->stream, F->d_int, F->n_int);
      }
      faces_join(c, F);
      {
        Prof p(c, "resid_restrict", (double)F->n_bnd * F->nc * F->nc * F->nc, lvl);
        launch_resid_restrict(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, nullptr, 1, F->d_parent_local,
                              F->d_dix, c->stream, F->d_bnd, F->n_bnd);
      }
    } else {
      Prof p(c, "resid_restrict", (double)F->n * F->nc * F->nc * F->nc, lvl);
      launch_resid_restrict(F->sweep_view(), view_of(c, lvl - 1), c->op, c->lambda, nullptr, 1, F->d_parent_local,
                            F->d_dix, c->stream);
    }
    restrict_remote(c, 1, lvl);
    restrict_remote(c, 4, lvl);
    // the fused step leaves the colour-1 halves of physical / refinement-
    // boundary ghosts as they were before the substep (k_smooth_resid); the
    // up-step's correction forms them again before anything reads them
    if (fused && (F->any_phys || F->any_rb)) F->phi_gc_ok = false;
  } else {
    residual_lvl(c, lvl, nullptr);
    restrict_lvl(c, 1, lvl);
    restrict_lvl(c, 4, lvl);
  }
  if (tail_crhs) return;
  Level* C = level_ptr(c, lvl - 1);
  // the fill of lvl-1 and its parents' coarse rhs in one pass when its faces
  // are same-GPU or physical (k_fill_crhs: a parent box reads its
  // neighbours' boundary cells itself instead of waiting for their pushes)
  if (C && C->n && !C->parents.empty() && !C->has_rb && !C->has_remote && !c->no_fill_tile && !c->no_fill_crhs &&
      (C->nc == 16 || C->nc == 8 || C->nc == 4)) {
    C->phi_gc_ok = true;
    rb_stale_above(c, lvl - 1);
    {
      Prof p(c, "fill_crhs", (double)C->n * C->nc * C->nc * C->nc, lvl - 1);
      launch_fill_crhs(C->sweep_view(), c->op, c->lambda, bc_for(c, lvl - 1, 1), C->d_parmask, c->stream);
    }
    finish_halo(c, C, 1);
    return;
  }
  fill_gc_lvl(c, lvl - 1, 1);
  if (C && !C->parents.empty()) {
    Prof p(c, "coarse_rhs", (double)C->parents.size() * C->nc * C->nc * C->nc, lvl - 1);
    if (!launch_coarse_rhs_tile(C->sweep_view(), c->op, c->lambda, C->d_parents, (int)C->parents.size(), c->stream))
      launch_coarse_rhs(C->view(), c->op, c->lambda, C->d_parents, (int)C->parents.size(), c->stream);
  }
}

// correct_children (m_multigrid.f90:387-402)
void correct_children(omg_ctx* c, int lvl) {
  Level* C = level_ptr(c, lvl);
  if (C && !C->parents.empty()) {
    Prof p(c, "sub_parents", (double)C->parents.size() * C->nc * C->nc * C->nc, lvl);
    launch_sub_parents(C->view(), C->d_parents, (int)C->parents.size(), c->stream);
  }
  prolong(c, lvl, 4, 1, 1);
}

// correct_children(lvl) + fill of lvl+1 + its first up-smoothing substep in
// one pass (k_prolong_smooth), when the level allows; returns whether it ran
// (the caller then starts smooth_boxes at substep 2).
bool prolong_smooth(omg_ctx* c, int lvl) {
  Level* F = level_ptr(c, lvl + 1);
  Level* C = level_ptr(c, lvl);
  // refinement-boundary faces: their coarse boxes on this GPU (decided alike
  // on every rank: any_rbx), formed on the device (no host refinement_bnd
  // for phi), 16^3 / 8^3 boxes
  const bool rb_ok = F && !c->no_rb_fill_fuse && !F->any_rbx && (F->nc == 16 || F->nc == 8) &&
                     !(F->rbh.count(1) && F->rbh.at(1).n);
  if (c->no_fuse_up || !F || !C || !F->prolong_smooth_ok || c->smoother != OMG_SMOOTHER_GSRB ||
      (c->op != OP_LPL && c->op != OP_HELM) ||
      c->n_cycle_up < 1 || (F->has_rb && !rb_ok) || (F->has_remote && !F->n_int) || !gs_tiled(F->nc, c->op, F->has_rb) ||
      !((size_t)F->n == 8 * C->parents.size() || C->nc * 2 == F->nc) ||
      (c->n_ranks > 1 && (F->prol.n_send || F->prol.n_recv)))
    return false;
  if (F->shift_pending) materialize_level(c, F);
  rb_stale_above(c, lvl + 1);
  const bool split = F->has_remote;
  {
    const int n = split ? F->n_int : F->n;
    Prof p(c, "prolong_smooth", (double)n * F->nc * F->nc * F->nc, lvl + 1);
    launch_prolong_smooth(C->view(), F->sweep_view(), c->op, c->lambda, F->d_parent_local, F->d_dix,
                          bc_for(c, lvl + 1, 1), C->nc * 2 == F->nc, split ? F->d_int : nullptr, n,
                          split ? F->d_push0 : nullptr, c->stream, F->has_rb, F->has_rb ? F->d_rbgv : nullptr);
    if (F->has_rb && F->d_rbgv) F->rbgv_ok = true;   // (its substep stored the coarse parts)
  }
  if (split) {
    // multi-GPU: boxes with a face on another GPU take the unfused pair,
    // correct + fill (their faces travel), then the colour-1 substep; their
    // same-GPU neighbours above pushed them the corrected colour 0 (push0)
    {
      Prof p(c, "prolong_fill", (double)F->n_bnd * F->nc * F->nc * F->nc, lvl + 1);
      launch_prolong_fill(C->view(), F->sweep_view(), 4, F->d_parent_local, F->d_dix, bc_for(c, lvl + 1, 1),
                          F->d_sendbuf, true, !c->no_skip1, c->stream, F->d_bnd, F->n_bnd, false,
                          F->h_rb.empty() ? nullptr : F->d_rb);
    }
    finish_halo(c, F, 1);
    {
      // (the boundary boxes' refinement-boundary coarse parts are stored here,
      // the interior boxes' by k_prolong_smooth: the level's whole buffer is
      // current after this)
      Prof p(c, "smoother_gsrb", 0.5 * F->n_bnd * F->nc * F->nc * F->nc, lvl + 1);
      launch_gs_substep(F->view(), c->op, c->lambda, 1, 1 << 1, view_of(c, lvl), F->d_rb, F->has_rb,
                        bc_for(c, lvl + 1, 1), F->d_sendbuf, nullptr, c->stream, F->d_bnd, F->n_bnd,
                        F->has_rb ? F->d_rbgv : nullptr, F->has_rb && F->d_rbgv ? 1 : 0);
    }
    finish_halo(c, F, 1);
  }
  // colour-0 ghost halves hold pre-correction values, but the next substep
  // reads only colour 1 and pushes colour 0 itself
  F->phi_gc_ok = true;
  return true;
}

// correct_children(l-1) + fill of l + up-smoothing substeps 1-3 of l in one
// k_gsrb3 pass (its correct_children form); returns whether it ran (the caller
// then starts smooth_boxes at substep 4).  Levels with k_gsrb3's coarse
// records (build_block3c), whose coarse level has consistent ghosts (the
// reference's correction reads the parents' ghost cells; the pass reads the
// neighbour parents' cells).
bool block3c_ok(omg_ctx* c, const Level* F) {
  return F && F->d_b3c && !c->no_block3 && !c->no_block3p && c->smoother == OMG_SMOOTHER_GSRB &&
         gsrb3_op_ok(c->op) && c->n_cycle_up * c->n_substeps >= 3;
}
// res_ready: the coarse level's last up pass stored its res = phi - old
// (smooth_boxes' want_res), which the pass then reads instead of phi and old;
// then, where the up-smoothing has four substeps or more, the pass is
// k_gsrb4's correction form, substeps 1-4 (round 6: level 1 of C3 815 + 308
// us for k_gsrb3's form + the one-substep launch before; OMG_NO_BLOCK4P: those)
// Returns the substeps run (0: none, the caller corrects otherwise).
int correct_block3(omg_ctx* c, int l, bool res_ready, bool defer_gc = false) {
  Level* F = level_ptr(c, l);
  Level* C = level_ptr(c, l - 1);
  if (!block3c_ok(c, F) || !C || !C->phi_gc_ok || C->shift_pending) return 0;
  // (a split level: only from the coarse res, whose proxies deep_res filled)
  if (F->deep && !res_ready) return 0;
  if (F->shift_pending) materialize_level(c, F);
  rb_stale_above(c, l);
  double* other = F->d_phi == F->d_data ? F->d_phi_buf : F->d_data;
  const LevelView cv = C->view();
  int done = 3;
  deep_before(c, F, 0);   // (the pass reads colour 0, before the correction)
  // defer_gc: nothing reads the level's ghosts before its next pass, which
  // reads none (the stand-alone V-cycle's last pass on its top level, see
  // fas_vcycle): the pass writes the interior only (12 of the 44 KB it
  // writes per box are ghost faces), and the ghosts are filled if anything
  // else comes first (Level::gc_deferred)
  bool deferred = false;
  if (res_ready && c->block4 && !c->no_block4p && c->n_cycle_up * c->n_substeps >= 4) {
    // (one rank: every rank decides its fills alike, see fas_vcycle)
    deferred = defer_gc && c->n_ranks == 1 && c->n_cycle_up * c->n_substeps == 4 && !F->deep && !F->b3_phys &&
               !c->no_defer_gc;
    Prof p(c, "smoother_gsrb4p", 2.0 * F->n * F->nc * F->nc * F->nc, l);
    launch_gsrb4(F->view(), other, F->d_b3, F->n_b3, c->op, c->lambda, 1, nullptr, c->stream, &cv, F->d_b3c,
                 nullptr, !deferred);
    done = 4;
  } else {
    Prof p(c, "smoother_gsrb3p", 1.5 * F->n * F->nc * F->nc * F->nc, l);
    launch_gsrb3(F->view(), other, F->d_b3, F->n_b3, c->op, c->lambda, 1, nullptr, c->stream, true, &cv, F->d_b3c,
                 res_ready ? 2 : 1);
  }
  F->d_phi = other;
  deep_after(c, F);
  F->phi_gc_ok = !deferred;
  F->gc_deferred = deferred;
  return done;
}

// correct_children(lvl) followed by mg_fill_ghost_cells_lvl(lvl+1, phi), as the
// V-cycle and FMG run them (m_multigrid.f90:127-136, 216-219); fused when every
// box of lvl+1 has its parent on this GPU (refinement-boundary ghosts are
// interpolated in the same kernel from lvl, which is final by then).
// then_gsrb: the caller smooths lvl+1 with red-black substeps right after
// (colour 1 first), so colour 1's correction is dead where no face needs it.
// save_old (FMG, fused path only, see correct_fill_fused): old = phi of lvl+1
// before the correction, the interior written by the fused kernel.
bool correct_fill_fused(omg_ctx* c, int lvl) {
  Level* F = level_ptr(c, lvl + 1);
  Level* C = level_ptr(c, lvl);
  return F && C && F->n && F->n_pairs == F->n && tiled_nc(F->nc) && !(F->has_rb && c->no_rb_fill_fuse) &&
         !(c->n_ranks > 1 && (F->prol.n_send || F->prol.n_recv));
}

void correct_and_fill(omg_ctx* c, int lvl, bool then_gsrb = false, bool save_old = false) {
  Level* F = level_ptr(c, lvl + 1);
  Level* C = level_ptr(c, lvl);
  if (save_old && (then_gsrb || !correct_fill_fused(c, lvl)))
    throw OmgError("internal: old = phi fused into an unfused correction");
  rb_stale_above(c, lvl + 1);
  if (correct_fill_fused(c, lvl)) {
    // every parent here has all its children on this GPU (no prolongation
    // traffic, every fine box has a local parent): the children form res
    const bool sub = (size_t)F->n == 8 * C->parents.size() || C->nc * 2 == F->nc;
    if (!sub && !C->parents.empty()) {
      Prof p(c, "sub_parents", (double)C->parents.size() * C->nc * C->nc * C->nc, lvl);
      launch_sub_parents(C->view(), C->d_parents, (int)C->parents.size(), c->stream);
    }
    {
      Prof p(c, "prolong_fill", (double)F->n * F->nc * F->nc * F->nc, lvl + 1);
      launch_prolong_fill(C->view(), F->sweep_view(), 4, F->d_parent_local, F->d_dix, bc_for(c, lvl + 1, 1),
                          F->d_sendbuf, sub, then_gsrb && !c->no_skip1, c->stream, nullptr, 0, save_old,
                          F->h_rb.empty() ? nullptr : F->d_rb);
    }
    finish_halo(c, F, 1);
    F->phi_gc_ok = true;
    return;
  }
  correct_children(c, lvl);
  fill_gc_lvl(c, lvl + 1, 1);
}

// MPI_Allreduce of one double: max exactly; sum in the recursive-doubling
// pairwise order of MPICH for power-of-two communicators.
double allreduce(omg_ctx* c, double v, bool is_max) {
  if (c->n_ranks == 1) return v;
  std::vector<double> all(c->n_ranks);
  if (c->loop) {
    all = loop_allgather(c, v);
  } else if (c->host_xport) {
    all = host_allgather(c, v);
  } else {
    double* d = c->d_scalar + 8;
    c->h_scalar[1] = v;
    HIPCHK(hipMemcpyAsync(d, &c->h_scalar[1], 8, hipMemcpyHostToDevice, c->stream));
    NCCLCHK(ncclAllGather(d, d + 1, 1, ncclDouble, (ncclComm_t)c->nccl, c->stream));
    HIPCHK(hipMemcpyAsync(all.data(), d + 1, 8 * c->n_ranks, hipMemcpyDeviceToHost, c->stream));
    host_sync(c, c->stream);
  }
  if (is_max) {
    // the device max is on IEEE bits (amax): NaN and Inf propagate; so must
    // the combination over ranks (std::max_element skips a NaN past all[0])
    double m = all[0];
    for (double x : all) {
      if (std::isnan(x)) return x;
      m = x > m ? x : m;
    }
    return m;
  }
  // MPI_Allreduce(MPI_SUM) as MPICH 3.3.2 computes it on one node
  // (m_multigrid.f90:255): a binomial-tree reduce to rank 0 in rank order,
  // ((a0+a1)+(a2+a3))+a4 ..., then a broadcast.  Pinned by the golden runs
  // of the reference at 1-6 and 8 ranks (per32_gsrb_v).
  for (int w = 1; w < c->n_ranks; w *= 2)
    for (int r = 0; r + w < c->n_ranks; r += 2 * w) all[r] = all[r] + all[r + w];
  return all[0];
}

// ---------------------------------------------------------------------------
// get_sum / subtract_mean on the device.  d_red slots: kAcc (this rank's sum,
// per channel phi / rhs), kMean (the mean), kAll (the gathered per-rank sums).
enum { kChPhi = 0, kChRhs = 1 };
double* red_acc(omg_ctx* c, int ch) { return c->d_red + ch; }
double* red_mean(omg_ctx* c, int ch) { return c->d_red + 2 + ch; }
double* red_all(omg_ctx* c, int ch) { return c->d_red + 8 + (size_t)ch * c->n_ranks; }

// get_sum's loop (m_multigrid.f90:278-294) for this rank, in two parts: the
// per-leaf sums of every level (into the channel's scratch), then acc = 0 and
// the sequential chains level by level.  Scratch and acc of a channel may be
// in use by a chain on the side stream: writers wait for it first.
double* leaf_scratch(Level* L, int ch) { return ch == kChRhs ? L->d_scratch_rhs : L->d_scratch; }

void side_done(omg_ctx* c) {
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_side, 0));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_phi, 0));
}

void leaf_box_sums(omg_ctx* c, int iv, int ch, hipStream_t st) {
  for (int l = 1; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    if (!L || L->leaves.empty()) continue;
    Prof p(c, "box_sums", (double)L->leaves.size() * L->nc * L->nc * L->nc, l, st);
    launch_box_sums(L->sweep_view(), iv, L->d_leaves, (int)L->leaves.size(), leaf_scratch(L, ch), st);
  }
}

void leaf_chain(omg_ctx* c, int ch, hipStream_t st) {
  double* acc = red_acc(c, ch);
  bool first = true;   // get_sum = 0 (:283): the first chain starts from +0.0 itself
  for (int l = 1; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    if (!L || L->leaves.empty()) continue;
    Prof p(c, "seq_sum", (double)L->leaves.size(), l, st);   // (timed on the stream it runs on)
    launch_seq_sum(leaf_scratch(L, ch), (int)L->leaves.size(), L->dr[0] * L->dr[1] * L->dr[2], acc, first, st);
    first = false;
  }
  if (first) HIPCHK(hipMemsetAsync(acc, 0, 8, st));
}

void leaf_sum_device(omg_ctx* c, int iv, int ch) {
  side_done(c);
  leaf_box_sums(c, iv, ch, c->stream);
  leaf_chain(c, ch, c->stream);
}

double subtract_volume(omg_ctx* c) {
  const int nc = c->box_size;
  const auto& d1 = c->drl[1];
  return (double)(nc * nc * nc) * (d1[0] * d1[1] * d1[2]) * (double)c->ids[1].size();
}

// MPI_Allreduce(acc) / volume into red_mean(ch), without leaving the stream
// (RCCL all-gather + k_mean); the loopback transport gathers on the host.
void mean_device(omg_ctx* c, int ch) {
  const int n = c->n_ranks;
  if (n > 64) throw OmgError("subtract_mean: more than 64 ranks");
  double* all = red_all(c, ch);
  if (n == 1) {
    all = red_acc(c, ch);
  } else if (c->loop || c->host_xport) {
    HIPCHK(hipMemcpyAsync(c->h_scalar + 4, red_acc(c, ch), 8, hipMemcpyDeviceToHost, c->stream));
    host_sync(c, c->stream);
    std::vector<double> v = c->loop ? loop_allgather(c, c->h_scalar[4]) : host_allgather(c, c->h_scalar[4]);
    for (int r = 0; r < n; r++) c->h_scalar[8 + r] = v[r];
    HIPCHK(hipMemcpyAsync(all, c->h_scalar + 8, 8 * n, hipMemcpyHostToDevice, c->stream));
  } else {
    NCCLCHK(ncclAllGather(red_acc(c, ch), all, 1, ncclDouble, (ncclComm_t)c->nccl, c->stream));
  }
  launch_mean(all, n, subtract_volume(c), red_mean(c, ch), c->stream);
}

// get_sum + MPI_Allreduce(sum) as one value on the host (omg_get_sum)
double get_sum(omg_ctx* c, int iv) {
  leaf_sum_device(c, iv, kChPhi);
  HIPCHK(hipMemcpyAsync(c->h_scalar + 2, red_acc(c, kChPhi), 8, hipMemcpyDeviceToHost, c->stream));
  host_sync(c, c->stream);
  return allreduce(c, c->h_scalar[2], false);
}

// The phi mean of a stand-alone cycle's subtract_mean is finished on the side
// stream (its chain overlaps the next cycle's rhs work); consumers wait here.
void phi_mean_ready(omg_ctx* c) {
  if (!c->phi_mean_on_side) return;
  c->phi_mean_on_side = false;
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_phi, 0));
  if (c->n_ranks > 1) mean_device(c, kChPhi);
}

// A pending phi -= mean (left by a standalone V-cycle, see subtract_mean) is
// applied before anything else reads phi.
void materialize_level(omg_ctx* c, Level* L) {
  if (!L->shift_pending) return;
  phi_mean_ready(c);
  L->shift_pending = false;
  rb_stale_above(c, L->lvl);
  if (L->n) {
    Prof p(c, "subtract", (double)L->n * L->nc * L->nc * L->nc, L->lvl);
    launch_subtract(L->view(), 1, red_mean(c, kChPhi), 1, c->stream);
  }
}
void materialize_phi(omg_ctx* c) {
  if (!c->phi_shift_pending) return;
  for (auto& kv : c->levels) materialize_level(c, &kv.second);
  c->phi_shift_pending = false;
}
// the ring-order rhs copies: every write of a level's rhs drops its copy
void drop_rhs_lex(omg_ctx* c) {
  for (auto& kv : c->levels) kv.second.rhs_lex_ok = kv.second.prox_rhs_ok = false;
}
// ring-order rhs buffers for the levels the register-ring lexicographic
// kernel serves (allocated outside any graph capture: tree setup, smoother
// choice): 16^3 levels large enough that the sweep is bandwidth-bound; on
// smaller levels the per-cycle copies cost more than they save (rings on
// levels of >= 512 or >= 64 boxes: 0.2-2 % slower, profiles/r03/s16,
// r04/s10_gs_ring_min_ab.txt)
constexpr int kGsRingMinBoxes = 2048;
// Called whenever the smoother or the operator changes (never inside a
// capture): the buffers exist exactly on the levels the current methods use
// them on, and are freed otherwise (a 512^3 level's are ~1.1 GiB).
void ensure_rhs_lex(omg_ctx* c) {
  if (c->host_only) return;
  const bool want = c->smoother != OMG_SMOOTHER_GSRB && !c->no_gs_plane;
  for (auto& kv : c->levels) {
    Level& L = kv.second;
    if (!want || L.n < kGsRingMinBoxes || !gs_lex_ring_ok(L.nc, c->op)) {
      if (L.d_rhs_lex || L.d_xlay) HIPCHK(hipStreamSynchronize(c->stream));   // (in use by queued sweeps)
      dfree(L.d_rhs_lex);
      dfree(L.d_xlay);
      dfree(L.d_galt);
      L.rhs_lex_ok = false;
      continue;
    }
    if (L.d_rhs_lex) continue;
    dmalloc(&L.d_rhs_lex, sizeof(double) * L.n * L.nc * L.nc * L.nc);
    dmalloc(&L.d_xlay, sizeof(double) * L.n * 2 * L.nc * L.nc);
    // the two-ghost-set chains skip the fills between sweeps, so only where
    // those fills exchange nothing: no remote or refinement-boundary faces,
    // and no coarse faces owed to another rank's refinement boundaries
    // (rbx.n_send: their fill_gc_lvl calls finish_rb after every sweep)
    if (!L.has_remote && !L.has_rb && L.rbx.n_send == 0 && L.rbx.n_recv == 0)
      dmalloc(&L.d_galt, sizeof(double) * L.n * 6 * (size_t)stored_face(L.nc));
    L.rhs_lex_ok = false;
  }
}
void drop_rhs_cache(omg_ctx* c) {
  c->rhs_cache_valid = false;
  drop_rhs_lex(c);
}
// entry points other than the cycles: apply pending phi work first; `writes`
// = the call may change rhs (the cached rhs sum is dropped)
void fill_gc_lvl(omg_ctx* c, int lvl, int iv);
void enter(omg_ctx* c, bool writes = true) {
  materialize_phi(c);
  for (auto& kv : c->levels)
    if (kv.second.gc_deferred) fill_gc_lvl(c, kv.first, 1);
  if (writes) drop_rhs_cache(c);
}

// subtract_mean (m_multigrid.f90:245-276), mean computed on the device.
// mode kInCycle: the standalone V-cycle's calls, where the next reads are
// known: rhs of levels whose boxes are all parents is overwritten by
// update_coarse before it is read (skipped), and phi -= mean is left pending:
// the first red-black substep of the next cycle subtracts it while loading
// (bit-identical), levels that restriction overwrites drop it, anything else
// applies it first (materialize_phi).
enum { kPlain = 0, kInCycle = 1 };
void subtract_mean(omg_ctx* c, int iv, int ghosts, int mode = kPlain) {
  // subtracting from interior and ghosts keeps same-GPU / remote face ghosts
  // equal to a fill; physical and refinement-boundary ghosts are not.
  if (iv == 1) {
    materialize_phi(c);
    for (auto& kv : c->levels)
      if (!ghosts || kv.second.any_phys || kv.second.any_rb) kv.second.phi_gc_ok = false;
  }
  if (iv == 2 && !ghosts) {
    // rhs: the sums may already be running on the side stream (see below)
    if (c->rhs_cache_valid) {
      HIPCHK(hipStreamWaitEvent(c->stream, c->ev_side, 0));
    } else {
      leaf_sum_device(c, 2, kChRhs);
    }
    c->rhs_cache_valid = false;
    // (split levels: proxies whose rhs was the owners' take the same
    // subtraction, bit for bit the owners' rhs - mean, and stay valid)
    std::vector<int> prox_kept;
    for (auto& kv : c->levels)
      if (kv.second.prox_rhs_ok) prox_kept.push_back(kv.first);
    drop_rhs_lex(c);
    mean_device(c, kChRhs);
    bool all_fused = true;
    for (int l = c->lowest; l <= c->highest; l++) {
      Level* L = level_ptr(c, l);
      if (!L || !L->n) continue;
      if (mode == kInCycle && L->all_parents) continue;
      if (L->n_prox && std::count(prox_kept.begin(), prox_kept.end(), l)) {
        LevelView P = L->view();   // the proxies as boxes 0 .. n_prox-1
        P.data += (long long)L->n * L->stride;
        P.phi += (long long)L->n * L->stride;
        P.n = L->n_prox;
        launch_subtract(P, 2, red_mean(c, kChRhs), 0, c->stream);
        L->prox_rhs_ok = true;
      }
      Prof p(c, "subtract_rhs", (double)L->n * L->nc * L->nc * L->nc, l);
      if (l >= 1 && (int)L->leaves.size() == L->n && subtract_sums_nc(L->nc))
        launch_subtract_sums(L->sweep_view(), 2, L->d_leaves, L->n, red_mean(c, kChRhs), L->d_scratch_rhs, c->stream);
      else {
        launch_subtract(L->view(), 2, red_mean(c, kChRhs), 0, c->stream);
        if (l >= 1 && !L->leaves.empty()) all_fused = false;
      }
    }
    if (all_fused) {
      // the next get_sum(rhs): its leaf sums were produced by the fused
      // kernels; its sequential chain runs now on the side stream
      HIPCHK(hipEventRecord(c->ev_main, c->stream));
      HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_main, 0));
      leaf_chain(c, kChRhs, c->stream2);
      HIPCHK(hipEventRecord(c->ev_side, c->stream2));
      c->rhs_cache_valid = true;
    }
    return;
  }
  if (iv == 2) drop_rhs_cache(c);
  const int ch = iv == 2 ? kChRhs : kChPhi;
  if (iv == 1 && ghosts && mode == kInCycle) {
    // leaf sums now, chain (+ mean on one rank) on the side stream; the next
    // cycle's rhs work overlaps it and phi_mean_ready() joins before use
    side_done(c);
    leaf_box_sums(c, 1, kChPhi, c->stream);
    HIPCHK(hipEventRecord(c->ev_main, c->stream));
    HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_main, 0));
    leaf_chain(c, kChPhi, c->stream2);
    if (c->n_ranks == 1) launch_mean(red_acc(c, kChPhi), 1, subtract_volume(c), red_mean(c, kChPhi), c->stream2);
    HIPCHK(hipEventRecord(c->ev_phi, c->stream2));
    c->phi_mean_on_side = true;
    for (auto& kv : c->levels) kv.second.shift_pending = kv.second.n > 0;
    c->phi_shift_pending = true;
    return;
  }
  leaf_sum_device(c, iv, ch);
  mean_device(c, ch);
  for (int l = c->lowest; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    if (L && L->n) {
      Prof p(c, "subtract", (double)L->n * L->nc * L->nc * L->nc, l);
      launch_subtract(L->view(), iv, red_mean(c, ch), ghosts, c->stream);
    }
  }
}

// The highest level `top` such that every level lowest..top can run inside
// the single-workgroup coarse program (launch_coarse_tail): a few boxes, all
// on this GPU, LDS-tiled box size, no refinement boundary, and every parent
// with all its children here.  INT_MIN when not even the lowest level can.
int tail_top(omg_ctx* c, int max_lvl) {
  // (the variable-coefficient operators measured faster level by level:
  // their single-workgroup program spills heavily)
  if (c->op != OP_LPL && c->op != OP_HELM) return INT_MIN;
  if (max_lvl - c->lowest + 1 > kTailMaxLevels) max_lvl = c->lowest + kTailMaxLevels - 1;
  int top = INT_MIN;
  for (int l = c->lowest; l <= max_lvl; l++) {
    Level* L = level_ptr(c, l);
    if (!L || L->n < 1 || L->n > kTailMaxBoxes || L->n != (int)c->ids[l].size() || L->has_rb ||
        !tiled_nc(L->nc))
      break;
    if (l > c->lowest) {
      Level* C = level_ptr(c, l - 1);
      if (L->n_pairs != L->n || !((size_t)L->n == 8 * C->parents.size() || C->nc * 2 == L->nc)) break;
    }
    top = l;
  }
  return top;
}

// Levels lowest..top of the V-cycle (down-smoothing of top .. up-smoothing of
// top) in one launch, bit-identical to the level-by-level path.
// the LDS-resident part of the tail (omg_tiles.hip): one box per level whose
// faces are physical or the box itself, the lowest levels up to 8^3 cells
// (at most three: 2^3, 4^3, 8^3, 5,120 doubles for their four variables),
// and a 16^3 top level right above them
void tail_lds_plan(omg_ctx* c, int top, int* lds_levels, int* lds_top) {
  const int n_lvls = top - c->lowest + 1;
  auto lds_box_ok = [&](int l, int max_nc) {
    Level* L = level_ptr(c, l);
    if (!L || L->n != 1 || L->nc > max_nc) return false;
    for (int nb = 0; nb < 6; nb++) {
      const int k = L->h_nbk[nb];
      if (!(k == NB_PHYS || (k == NB_LOCAL && L->h_nba[nb] == 0))) return false;
    }
    return true;
  };
  int n = 0;
  while (n < std::min(n_lvls, kTailLdsMaxLevels) && lds_box_ok(c->lowest + n, 8)) n++;
  *lds_levels = n;
  *lds_top = n > 0 && n == n_lvls - 1 && level_ptr(c, top)->nc == 16 && lds_box_ok(top, 16);
}

// whether the tail can take over update_coarse's fill and coarse rhs of its
// top level: a single parent box on this GPU whose faces are physical or same-
// GPU (kTailMaxBoxes), after a level-by-level down-step of top+1
bool tail_crhs_ok(omg_ctx* c, int top) {
  const Level* T = level_ptr(c, top);
  return !c->no_tail_crhs && T && T->n == 1 && !T->parents.empty() && !T->has_rb && !T->has_remote &&
         level_ptr(c, top + 1) != nullptr;
}

void run_tail(omg_ctx* c, int top, bool top_crhs) {
  TailArgs A;
  std::memset(&A, 0, sizeof(A));   // padding too: compared bytewise below
  A.n_lvls = top - c->lowest + 1;
  for (int l = c->lowest; l <= top; l++) {
    Level* L = level_ptr(c, l);
    if (L->shift_pending) {
      if (L->all_parents && l < top) L->shift_pending = false;   // overwritten by the restriction
      else materialize_level(c, L);
    }
    L->rhs_lex_ok = L->prox_rhs_ok = false;   // the tail writes the rhs of the levels below its top
    TailLevel& T = A.lv[l - c->lowest];
    T.L = L->view();
    T.bc = bc_for(c, l, 1);
    T.parents = L->d_parents;
    T.n_par = (int)L->parents.size();
    T.parent_local = L->d_parent_local;
    T.dixp = L->d_dix;
    // the first box's bc table entries inline (the LDS setup reads them
    // without a dependent load)
    auto fo = c->h_face_off_lvl[0].find(l);
    auto ft = c->h_face_type_lvl[0].find(l);
    for (int nb = 0; nb < 6; nb++) {
      const bool tab = fo != c->h_face_off_lvl[0].end() && fo->second.size() >= 6;
      const long long o = tab ? fo->second[nb] : -1;
      T.foff[nb] = o > INT_MAX ? -2 : (int)o;
      T.ftype[nb] = (signed char)(tab && ft != c->h_face_type_lvl[0].end() && ft->second.size() >= 6 ? ft->second[nb] : 0);
    }
  }
  A.lambda = c->lambda;
  A.n_down = c->n_cycle_down;
  A.n_up = c->n_cycle_up;
  A.max_coarse = c->max_coarse_cycles;
  A.res_abs = c->res_abs;
  A.res_rel = c->res_rel;
  A.maxbits = (unsigned long long*)c->d_scalar;
  A.coarse_its = (int*)(c->d_scalar + 1);
  A.gs_lex = c->smoother != OMG_SMOOTHER_GSRB;
  A.top_crhs = top_crhs;
  tail_lds_plan(c, top, &A.lds_levels, &A.lds_top);
  const bool tail_timing = c->tail_timing;
  if (tail_timing) {
    if (!c->d_tail_stamps) HIPCHK(hipMalloc(&c->d_tail_stamps, 8 * 64));   // (never captured: graph_ok)
    A.stamps = c->d_tail_stamps;
    HIPCHK(hipMemsetAsync(c->d_tail_stamps, 0, 8 * 64, c->stream));   // (unwritten stamps stay 0)
  }
  if (std::memcmp(&A, c->h_tail, sizeof(TailArgs)) != 0) {
    *c->h_tail = A;   // what d_tail holds once the stream gets here
    launch_store_tail(A, c->d_tail, c->stream);
  }
  {
    Prof p(c, "coarse_tail", 0.0, top);
    launch_coarse_tail(c->d_tail, A.gs_lex, c->op, c->stream);
  }
  if (tail_timing) {   // diagnostics: phase times of the tail (100 MHz wall clock)
    long long h[64];
    HIPCHK(hipMemcpyAsync(h, c->d_tail_stamps, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    host_sync(c, c->stream);
    std::fprintf(stderr, "tail us:");
    for (int i = 1; i < 64 && h[i]; i++) std::fprintf(stderr, " %.1f", (h[i] - h[i - 1]) * 0.01);
    std::fprintf(stderr, "\n");
  }
  for (int l = c->lowest; l <= top; l++) level_ptr(c, l)->phi_gc_ok = true;
  rb_stale_above(c, top);
}

// Failure detection: the device max residual is an exact max of
// |res| over IEEE bits, so one NaN or Inf cell makes it non-finite.  The
// reference's Fortran max() drops NaN operands (m_multigrid.f90:226-234,
// 296-311) and reports a finite or zero residual for a diverged field; here
// it is an error instead, the caller's output argument holding the bits.
void check_finite_res(double r, const char* where) {
  if (!std::isfinite(r))
    throw OmgError(std::string(where) + ": non-finite residual (" + (std::isnan(r) ? "NaN" : "Inf") +
                   "): phi or rhs holds NaN/Inf");
}

// mg_fas_vcycle (m_multigrid.f90:150-243)
double fas_vcycle(omg_ctx* c, int highest_lvl, bool want_max_res, bool standalone) {
  const bool has_highest = highest_lvl >= c->lowest;
  const int min_lvl = c->lowest, max_lvl = has_highest ? highest_lvl : c->highest;
  const bool full = standalone && !has_highest;   // a stand-alone cycle over the whole tree
  // a pending phi shift (previous stand-alone cycle) is absorbed by the first
  // substep on max_lvl or dropped where restriction overwrites a level
  if (c->phi_shift_pending) {
    if (!full) {
      materialize_phi(c);
    } else {
      for (auto& kv : c->levels) {
        Level& L = kv.second;
        if (L.shift_pending && L.lvl != max_lvl && !L.all_parents) materialize_level(c, &L);
      }
    }
  }
  if (c->subtract_mean && !has_highest) subtract_mean(c, 2, 0, full ? kInCycle : kPlain);
  if (standalone) {
    // the fill is idempotent: skip it when the ghosts already equal its result.
    // Fills exchange halos, so every rank must decide alike; the decision is
    // rank-invariant without communication: phi_gc_ok changes only in calls
    // every rank makes (fills, cycles, restriction / prolongation, collective
    // uploads of phi, see omg.h), and any_rb is a property of the global
    // tree.  (Agreeing over the transport instead, as round 3 did, cost a
    // host synchronisation per cycle.)  OMG_CHECK_COLLECTIVE checks it.
    // A level with refinement boundaries is consistent as long as the level
    // below was not written since its last fill (rb_stale_above).  With a
    // subtracted mean those writes depend on per-rank state (pending mean
    // shifts, materialised where a rank has boxes), so with more than one
    // rank such a level is then always refilled.
    Level* L = level_ptr(c, max_lvl);
    bool need = !(L && L->phi_gc_ok && (!L->any_rb || c->n_ranks == 1 || !c->subtract_mean));
    // (ghosts deferred by the last cycle: its first pass reads none, k_gsrb4 /
    // k_gsrb3, and writes them all; smooth_boxes fills first otherwise)
    if (L && L->gc_deferred && c->smoother == OMG_SMOOTHER_GSRB && tail_top(c, max_lvl) < max_lvl) need = false;
    if (c->n_ranks > 1 && c->check_collective && (allreduce(c, need ? 1.0 : 0.0, true) > 0.5) != need)
      throw OmgError("mg_fas_vcycle: the stand-alone fill decision differs across ranks "
                     "(an upload of phi was not made on every rank)");
    if (need) {
      if (L) materialize_level(c, L);
      fill_gc_lvl(c, max_lvl, 1);
    }
  }
  const int top = tail_top(c, max_lvl);
  const bool tail = top >= min_lvl && !c->no_tail;
  const bool tail_crhs = tail && max_lvl > top && tail_crhs_ok(c, top);
  for (int l = max_lvl; l >= min_lvl + 1; l--) {
    if (tail && l <= top) break;
    // four substeps per pass, then the unfused residual (k_resid_restrict):
    // C3 4.06 -> 3.97 ms against k_gsrb3 + k_smooth_resid (level 1 775 + 592
    // us; level 0 even, profiles/r05/s50_block4_ab.txt); OMG_NO_BLOCK4: the latter
    // (a level with physical faces: k_gsrb3 + k_smooth_resid, whose k_gsrb4
    // takes a workgroup per CU, 114 VGPRs; OMG_BLOCK4_PHYS: k_gsrb4 there too)
    B3Phys P3;
    const B3Phys* ph = nullptr;
    const bool four = c->block4 && c->smoother == OMG_SMOOTHER_GSRB && b3_usable(c, l, P3, ph) &&
                      (!ph || c->block4_phys) && (c->n_cycle_down * c->n_substeps) % 4 == 0;
    const bool fused = !four && smooth_resid_ok(c, l);
    // (the down pass writes its ghosts, which the residual reads: leaving them
    // to a residual that gathers the neighbours' boundary cells instead took
    // C3's down pass 837 -> 713 us and the residual 590 -> 750 us, the x faces'
    // cells 64 B apart in the neighbours' boxes; profiles/r06/s19_defer_down_ab.txt)
    smooth_boxes(c, l, c->n_cycle_down, 1, fused ? 1 : 0, false, four, four);
    update_coarse(c, l, fused, tail_crhs && l == top + 1);
    faces_join(c, level_ptr(c, l));   // (update_coarse joined them; defensive)
  }
  if (tail) {
    run_tail(c, top, tail_crhs);
  } else {
    // coarse grid: all its boxes live on one rank (error stop otherwise, :197-200)
    const auto& ids = c->ids[min_lvl];
    for (int id : ids)
      if (min_lvl > c->rep_lvl && c->rank_of[id - 1] != c->rank_of[ids[0] - 1])
        throw OmgError("Multiple CPUs for coarse grid (not implemented yet)");
    // a rank without the coarse boxes has nothing to do here: they all live on
    // one rank, so their smoothing exchanges nothing (the reference's other
    // ranks run empty loops until the owner's residual test, which they never
    // see either, m_multigrid.f90:202-208); skipping it saves them a host wait
    // per coarse sweep
    const Level* Lmin = level_ptr(c, min_lvl);
    const bool own_coarse = Lmin && Lmin->n > 0;
    double init_res = own_coarse ? max_residual_lvl(c, min_lvl) : 0.0;
    for (int i = 1; own_coarse && i <= c->max_coarse_cycles; i++) {
      smooth_boxes(c, min_lvl, c->n_cycle_up + c->n_cycle_down);
      double res = max_residual_lvl(c, min_lvl);
      if (res < c->res_rel * init_res || res < c->res_abs) break;
    }
  }
  // res_ready: level l-1's last up pass stored its res (correct_children's
  // phi - old) for level l's correct_children form.  A level whose level
  // above takes that form (want_res) ends its up-smoothing with that pass, so
  // it starts with k_prolong_smooth rather than the form itself (which leaves
  // a plain last substep).
  bool res_ready = false;
  for (int l = (tail ? top : min_lvl) + 1; l <= max_lvl; l++) {
    const bool want_res = l < max_lvl && block3c_ok(c, level_ptr(c, l + 1)) && !c->no_block3r;
    bool done = false;
    int pro = 0;
    if (!want_res && (pro = correct_block3(c, l, res_ready, full && l == max_lvl && !want_max_res)) > 0) {
      done = smooth_boxes(c, l, c->n_cycle_up, pro + 1);
    } else {
      // (the other correction paths read the level's ghosts: deferred ones are
      // filled first)
      if (Level* Fd = level_ptr(c, l); Fd && Fd->gc_deferred) fill_gc_lvl(c, l, 1);
      if (prolong_smooth(c, l - 1)) {
        done = smooth_boxes(c, l, c->n_cycle_up, 2, 0, want_res);
      } else {
        correct_and_fill(c, l - 1, c->smoother == OMG_SMOOTHER_GSRB && c->n_cycle_up >= 1);
        done = smooth_boxes(c, l, c->n_cycle_up, 1, 0, want_res);
      }
    }
    res_ready = done;
  }
  double max_res = 0.0;
  if (want_max_res) {
    double m = 0.0;
    if (min_lvl <= max_lvl) m = max_residual_levels(c, min_lvl, max_lvl);
    max_res = allreduce(c, m, true);
  }
  materialize_phi(c);   // nothing left pending after a cycle (defensive: all consumed)
  if (c->subtract_mean) subtract_mean(c, 1, 1, full ? kInCycle : kPlain);
  return max_res;
}

// mg_fas_fmg (m_multigrid.f90:84-147)
double fas_fmg(omg_ctx* c, bool have_guess, bool want_max_res) {
  if (have_guess) {
    materialize_phi(c);
  } else {
    for (auto& kv : c->levels) kv.second.shift_pending = false;   // phi = 0 below
    c->phi_shift_pending = false;
  }
  if (!have_guess) phi_dirty_all(c);
  if (!have_guess)
    for (int l = c->highest; l >= c->lowest; l--) {
      Level* L = level_ptr(c, l);
      if (L && L->n) launch_copy_var(L->view(), 0, 1, c->stream);
    }
  fill_gc_lvl(c, c->highest, 1);
  for (int l = c->highest; l >= c->lowest + 1; l--) update_coarse(c, l);
  if (c->subtract_mean) subtract_mean(c, 2, 0);
  double max_res = 0.0;
  for (int l = c->lowest; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    // old = phi (:127-129).  Below the highest level, where every box is a
    // parent, update_coarse's parent loop above left old equal to phi, ghost
    // faces included, and nothing has written that level since (unless the
    // cycles below subtract phi's mean, which covers every level)
    // Elsewhere the copy's interior half rides on the fused correction, which
    // loads the pre-correction interior anyway: only the ghost faces are copied
    const bool old_is_phi = l < c->highest && L && L->all_parents && !c->subtract_mean;
    const bool save_old = L && L->n && !old_is_phi && l > c->lowest && correct_fill_fused(c, l - 1);
    if (save_old) {
      launch_copy_ghosts(L->view(), c->stream);
    } else if (L && L->n && !old_is_phi) {
      launch_copy_var(L->view(), 1, 3, c->stream);
    }
    if (l > c->lowest) correct_and_fill(c, l - 1, false, save_old);
    if (l == c->highest)
      max_res = fas_vcycle(c, l, want_max_res, false);
    else
      fas_vcycle(c, l, false, false);
  }
  return max_res;
}

// A whole cycle (V-cycle or FMG) as one HIP graph: the host logic runs as
// usual while the stream is captured, so every kernel argument and every
// host-side state change is exactly that of the direct launches; the graph of
// the previous call with the same key is updated in place (same topology) or
// re-instantiated, then launched.  A graph issues a dependent kernel in ~1.8
// us of host time against ~3.2 us direct (tools/graph_probe.hip), but the
// cycles measured no faster (C1 0.252 -> 0.260 ms, C4 0.553 -> 0.568, 512^3
// FMG 11.65 -> 11.49): their small-level kernels are bound by their own
// 3-5 us on the GPU, not by the host, and capturing costs what it saves.
// Opt-in (OMG_GRAPH=1).  Only where the cycle never waits for the host:
// one GPU, no subtract_mean (its side-stream chain spans calls), every
// V-cycle ends in the coarse tail (the level-by-level coarse solve reads its
// residual back per sweep), no profiling.
bool graph_ok(omg_ctx* c) {
  return !c->no_graph && !c->capturing && c->n_ranks == 1 && !c->subtract_mean && !c->profiling && !c->rbh_any &&
         !c->tail_timing && !c->no_tail && c->n_boxes > 0 && tail_top(c, c->highest) >= c->lowest;
}

// The host state the captured body changed assumes the graph ran.  When the
// capture, instantiation or launch fails, that is rolled back to "unknown":
// the tail arguments are re-uploaded by the next call (h_tail no longer
// matches anything), the graph of this key is dropped, and every level's phi
// ghost faces count as stale (the next cycle fills them).  (The graph path
// runs without subtract_mean, so no mean / shift state is involved.)
void graph_rollback(omg_ctx* c, int key, const std::map<int, double*>& phi_at_start) {
  c->capturing = false;
  // the multi-substep passes swap a level's phi buffer on the host as they are
  // recorded: a graph that never ran leaves phi where it was
  for (auto& kv : phi_at_start) c->levels[kv.first].d_phi = kv.second;
  c->max_deferred = false;
  std::memset(c->h_tail, 0xff, sizeof(TailArgs));
  auto it = c->graphs.find(key);
  if (it != c->graphs.end()) {
    if (it->second) (void)hipGraphExecDestroy(it->second);
    c->graphs.erase(it);
  }
  phi_dirty_all(c);
  // the captured body may have recorded the ring-order rhs copy (and marked
  // it built) without the graph ever running
  drop_rhs_lex(c);
  (void)hipGetLastError();
}

template <typename F>
double run_cycle(omg_ctx* c, int key, F&& body) {
  if (!graph_ok(c)) return body();
  std::map<int, double*> phi_at_start;
  for (auto& kv : c->levels) phi_at_start[kv.first] = kv.second.d_phi;
  c->capturing = true;
  c->max_deferred = false;
  HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  hipGraph_t g = nullptr;
  try {
    if (c->graph_fail_at == 1) {   // one-shot test injection
      c->graph_fail_at = 0;
      throw OmgError("injected failure during capture (OMG_GRAPH_FAIL=1)");
    }
    body();
  } catch (...) {
    (void)hipStreamEndCapture(c->stream, &g);
    if (g) (void)hipGraphDestroy(g);
    graph_rollback(c, key, phi_at_start);
    throw;
  }
  c->capturing = false;
  try {
    HIPCHK(hipStreamEndCapture(c->stream, &g));
    size_t n_nodes = 0;
    HIPCHK(hipGraphGetNodes(g, nullptr, &n_nodes));
    if (c->graph_fail_at == 2) {   // one-shot: the body ran (host state changed), the graph does not
      c->graph_fail_at = 0;
      throw OmgError("injected failure before the launch (OMG_GRAPH_FAIL=2)");
    }
    if (n_nodes) {
      hipGraphExec_t& ex = c->graphs[key];
      if (ex) {
        hipGraphNode_t err_node = nullptr;
        hipGraphExecUpdateResult res;
        if (hipGraphExecUpdate(ex, g, &err_node, &res) != hipSuccess || res != hipGraphExecUpdateSuccess) {
          (void)hipGetLastError();
          HIPCHK(hipGraphExecDestroy(ex));
          ex = nullptr;
        }
      }
      if (!ex) HIPCHK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      HIPCHK(hipGraphLaunch(ex, c->stream));
    }
  } catch (...) {
    if (g) (void)hipGraphDestroy(g);
    graph_rollback(c, key, phi_at_start);
    throw;
  }
  HIPCHK(hipGraphDestroy(g));
  if (!c->max_deferred) return 0.0;
  c->max_deferred = false;
  host_sync(c, c->stream);
  return c->h_scalar[0];
}

// mg_set_methods' operator part + *_set_lambda (m_multigrid.f90:27-60,
// m_helmholtz.f90:39-46, m_vhelmholtz.f90:51-58, m_ahelmholtz.f90:59-66)
void set_operator(omg_ctx* c, int op, double lambda) {
  if (op < OMG_LAPLACIAN || op > OMG_AHELMHOLTZ) throw OmgError("mg_set_methods: unknown operator");
  if (lambda < 0) throw OmgError("helmholtz_set_lambda: lambda < 0 not allowed");
  if (op == OMG_AHELMHOLTZ && c->n_vars < 7 && c->n_boxes > 0)
    throw OmgError("ahelmholtz_set_methods: needs 3 extra variables");
  if ((op == OMG_VLAPLACIAN || op == OMG_VHELMHOLTZ) && c->n_vars < 5 && c->n_boxes > 0)
    throw OmgError("vlaplacian/vhelmholtz_set_methods: mg%n_extra_vars == 0");
  if (op == OMG_VLAPLACIAN) lambda = 0.0;
  const bool changed = c->op != op;
  c->op = op;
  c->lambda = lambda;
  if (changed && !c->capturing) ensure_rhs_lex(c);
}

// mg_apply_op (m_multigrid.f90:439-456): box_op on every box of every level
void apply_op(omg_ctx* c, int i_out) {
  enter(c);
  if (i_out == 1) phi_dirty_all(c);
  for (int l = c->lowest; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    if (L && L->n) launch_box_op(L->view(), c->op, c->lambda, i_out, c->stream);
  }
}

// m_diffusion's set_rhs (m_diffusion.f90:144-159): rhs = f1*phi + f2*rhs on
// the interior of this rank's leaves of levels 1..highest
void set_rhs(omg_ctx* c, double f1, double f2) {
  enter(c);
  for (int l = 1; l <= c->highest; l++) {
    Level* L = level_ptr(c, l);
    if (!L || L->leaves.empty()) continue;
    launch_set_rhs(L->view(), L->d_leaves, (int)L->leaves.size(), f1, f2, c->stream);
  }
}

// diffusion_solve / diffusion_solve_vcoeff / diffusion_solve_acoeff
// (m_diffusion.f90:19-57, :63-101, :108-142): one implicit time step of
// order 1 (backward Euler) or 2 (Crank-Nicolson) as a Helmholtz problem,
// FMG first, then up to 10 V-cycles until max_res.  The three differ only in
// the operator and in lambda = 1/(dt*D) vs 1/dt (D = 1 for the v/a forms).
constexpr int kDiffusionMaxIts = 10;   // m_diffusion.f90:25
void diffusion_solve(omg_ctx* c, int op, double dt, double coeff, int order, double max_res, int* n_vcycles,
                     double* res_out) {
  if (op != OMG_HELMHOLTZ && op != OMG_VHELMHOLTZ && op != OMG_AHELMHOLTZ)
    throw OmgError("diffusion_solve: operator must be helmholtz, vhelmholtz or ahelmholtz");
  if (order != 1 && order != 2) throw OmgError("diffusion_solve: order should be 1 or 2");
  const double dtc = op == OMG_HELMHOLTZ ? dt * coeff : dt;
  // helmholtz_set_methods / vhelmholtz_set_methods clear subtract_mean;
  // ahelmholtz_set_methods leaves it as it was
  set_operator(c, op, 0.0);
  if (op != OMG_AHELMHOLTZ) c->subtract_mean = 0;
  if (order == 1) {
    set_operator(c, op, 1 / dtc);
    set_rhs(c, -1 / dtc, 0.0);
  } else {
    apply_op(c, 2);   // lambda = 0: rhs = L(phi) on every level
    set_operator(c, op, 2 / dtc);
    set_rhs(c, -2 / dtc, -1.0);
  }
  double res = run_cycle(c, 2 + 2 + 4, [&] { return fas_fmg(c, true, true); });
  int n = 1;
  for (; n <= kDiffusionMaxIts; n++) {
    if (!std::isfinite(res)) {   // the outputs hold the state at the error (omg.h)
      if (n_vcycles) *n_vcycles = n - 1;
      if (res_out) *res_out = res;
      check_finite_res(res, "diffusion_solve");
    }
    if (res <= max_res) break;
    res = run_cycle(c, 1 + 2 + 4 + 8 * (c->lowest - 1 + 64),
                    [&] { return fas_vcycle(c, c->lowest - 1, true, true); });
  }
  if (n_vcycles) *n_vcycles = n - 1;
  if (res_out) *res_out = res;
  if (n == kDiffusionMaxIts + 1) throw OmgError("diffusion_solve: no convergence");
}

// ---------------------------------------------------------------------------
// mg_phi_bc_store (m_ghost_cells.f90:66-117): the bc values of phi go into
// the rhs ghost cells and the bc type into the neighbour slot.
void phi_bc_store(omg_ctx* c) {
  phi_dirty_all(c);
  for (auto& kv : c->levels) {
    Level& L = kv.second;
    if (!L.n) continue;
    GcBC g = bc_for(c, kv.first, 1);
    g.phi_stored = 0;
    launch_phi_bc_store(L.view(), g, L.d_nba, c->stream);
    HIPCHK(hipMemcpyAsync(L.h_nba.data(), L.d_nba, sizeof(int) * L.h_nba.size(), hipMemcpyDeviceToHost,
                          c->stream));
    host_sync(c, c->stream);
    for (int b = 0; b < L.n; b++)
      for (int nb = 1; nb <= 6; nb++)
        if (L.h_nbk[(size_t)b * 6 + nb - 1] == NB_PHYS)
          c->neighbors[(size_t)(L.ids[b] - 1) * 6 + nb - 1] = L.h_nba[(size_t)b * 6 + nb - 1];
    pack_topo(L);
  }
  c->phi_bc_data_stored = 1;
}

// ---------------------------------------------------------------------------
// Free-space boundary conditions: mg_poisson_free_3d (m_free_space.f90:36-214)
// with PSolver's solve on the device (omg_free.hip).

#define FFTCHK(x)                                                                          \
  do {                                                                                     \
    hipfftResult r_ = (x);                                                                 \
    if (r_ != HIPFFT_SUCCESS) throw OmgError(std::string(#x) + ": hipFFT error " + std::to_string((int)r_)); \
  } while (0)

// smallest even n >= m whose prime factors are 2, 3, 5, 7 (the transform
// length of one padded axis)
int fft_length(int m) {
  for (int n = std::max(m, 2);; n++) {
    if (n & 1) continue;
    int r = n;
    for (int f : {2, 3, 5, 7})
      while (r % f == 0) r /= f;
    if (r == 1) return n;
  }
}

void free_grid_release(omg_free_state* S) {
  dfree(S->d_R);
  dfree(S->d_Z);
  dfree(S->d_karray);
  dfree(S->d_planes);
  dfree(S->d_my);
  dfree(S->d_my_ix);
  dfree(S->d_send);
  dfree(S->d_recv);
  dfree(S->d_recv_ix);
  dfree(S->gather.d_send_items);
  dfree(S->gather.d_recv_items);
  S->gather = Transfer();
  if (S->have_plans) {
    (void)hipfftDestroy(S->fwd);
    (void)hipfftDestroy(S->inv);
    S->have_plans = false;
  }
  S->initialized = false;
  S->fft_lvl = INT_MIN;
}

void free_state_destroy(omg_ctx* c) {
  if (!c->free_state) return;
  free_grid_release(c->free_state);
  delete c->free_state;
  c->free_state = nullptr;
}

// createKernel(geocode 'F', nx(1), nx(3), nx(3), dr, itype_scf = 8)
// (m_free_space.f90:118-120, build_kernel.f90:55-199, 884-1164): the kernel
// spectrum * scal on the grid S->G.
void free_create_kernel(omg_ctx* c, omg_free_state* S, const double h[3]) {
  const FreeGrid& G = S->G;
  // the reference creates the kernel for (nx(1), nx(3), nx(3)); the extents
  // of the tables are the grid's own (equal whenever ny == nz)
  const int n0k[3] = {G.nx[0], G.nx[2], G.nx[2]};
  int n_range = 2 * kFreeItype;
  for (int d = 0; d < 3; d++) n_range = std::max(n_range, G.n0[d]);
  if (n_range > kFreeMaxRange) throw OmgError("mg_poisson_free_3d: FFT grid too large for the kernel tables");
  double a[3];
  for (int d = 0; d < 3; d++) a[d] = h[d] * (double)n0k[d];
  const double factor = 1.0 / std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  const double factor2 = 1.0 / (a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  const bool cube = h[0] == h[1] && h[1] == h[2];
  // per Gaussian in the order the reference sums them (i_gauss = 89 .. 1):
  // weight, starting exponent and number of scf_recursion passes per axis
  std::vector<double> w(kFreeNGauss), p0(3 * kFreeNGauss);
  std::vector<int> nit(3 * kFreeNGauss);
  for (int g = 0; g < kFreeNGauss; g++) {
    const int ig = kFreeNGauss - 1 - g;
    const double pg = factor2 * kGequadP[ig];
    w[g] = factor * kGequadW[ig];
    for (int d = 0; d < 3; d++) {
      const double pref = 1.0 / (cube ? h[0] * h[0] : h[d] * h[d]);
      long n = std::lround((std::log(pg) - std::log(pref)) / std::log(4.0));
      if (n <= 0) n = 0;
      nit[3 * g + d] = (int)n;
      p0[3 * g + d] = n == 0 ? pg : pg / std::pow(4.0, (double)n);
    }
  }
  int n0max = std::max(G.n0[0], std::max(G.n0[1], G.n0[2]));
  double *d_p0 = nullptr, *d_w = nullptr, *d_tab = nullptr, *d_work = nullptr, *d_F = nullptr;
  int* d_nit = nullptr;
  const int fmax = std::max(G.N[0], std::max(G.N[1], G.N[2])) / 2 + 1;
  d_p0 = to_device(p0);
  d_w = to_device(w);
  d_nit = to_device(nit);
  dmalloc(&d_tab, sizeof(double) * 3 * kFreeNGauss * (size_t)n0max, true);
  dmalloc(&d_work, sizeof(double) * 3 * kFreeNGauss * (size_t)(n_range + 1), true);
  dmalloc(&d_F, sizeof(double) * 3 * kFreeNGauss * (size_t)fmax, true);
  FreeTabArgs A;
  A.p0 = d_p0;
  A.n_iter = d_nit;
  for (int d = 0; d < 3; d++) {
    A.h[d] = cube ? h[0] : h[d];
    A.n0[d] = G.n0[d];
  }
  A.cube = cube;
  A.n_range = n_range;
  A.n0max = n0max;
  A.tab = d_tab;
  A.work = d_work;
  launch_free_tables(A, c->stream);
  launch_free_dft(d_tab, n0max, G, d_F, fmax, c->stream);
  const size_t nk = (size_t)(G.N[0] / 2 + 1) * G.N[1] * G.N[2];
  dmalloc(&S->d_karray, sizeof(double) * nk);
  // PSolver's scal = hx*hy*hz/(n1*n2*n3) (psolver_main.f90:297)
  const double scal = h[0] * h[1] * h[2] / ((double)G.N[0] * (double)G.N[1] * (double)G.N[2]);
  launch_free_karray(d_F, fmax, d_w, G, scal, S->d_karray, c->stream);
  host_sync(c, c->stream);
  dfree(d_p0);
  dfree(d_w);
  dfree(d_nit);
  dfree(d_tab);
  dfree(d_work);
  dfree(d_F);
}

// the FFT grid, its plans and the gather plan of the FFT level
void free_new_grid(omg_ctx* c, omg_free_state* S, int fft_lvl, const int nx[3], const double h[3]) {
  FreeGrid& G = S->G;
  // the density is zero on the ghost layer, so the offsets the solution
  // needs are |d| <= nx-2 and N >= 2*(nx-2) gives the linear convolution
  // (a power of two for power-of-two domains; the k_free_dft note)
  for (int d = 0; d < 3; d++) {
    G.nx[d] = nx[d];
    G.n0[d] = nx[d];
    G.N[d] = fft_length(std::max(2 * (nx[d] - 2), nx[d]));   // and the nx points fit
  }
  free_create_kernel(c, S, h);
  const size_t nr = (size_t)G.N[0] * G.N[1] * G.N[2], nz = (size_t)(G.N[0] / 2 + 1) * G.N[1] * G.N[2];
  dmalloc(&S->d_R, sizeof(double) * nr);
  dmalloc(&S->d_Z, sizeof(double2) * nz);
  dmalloc(&S->d_planes, sizeof(double) * 2 *
                            ((size_t)nx[1] * nx[2] + (size_t)nx[0] * nx[2] + (size_t)nx[0] * nx[1]));
  FFTCHK(hipfftPlan3d(&S->fwd, G.N[2], G.N[1], G.N[0], HIPFFT_D2Z));
  FFTCHK(hipfftPlan3d(&S->inv, G.N[2], G.N[1], G.N[0], HIPFFT_Z2D));
  S->have_plans = true;
  FFTCHK(hipfftSetStream(S->fwd, c->stream));
  FFTCHK(hipfftSetStream(S->inv, c->stream));
  // my boxes at the FFT level (a replicated level holds all of them)
  Level* L = level_ptr(c, fft_lvl);
  std::vector<int> my, my_ix;
  if (L)
    for (int b = 0; b < L->n; b++) {
      my.push_back(b);
      for (int d = 0; d < 3; d++) my_ix.push_back(c->ix[(size_t)(L->ids[b] - 1) * 3 + d]);
    }
  S->n_my = (int)my.size();
  S->d_my = to_device(my);
  S->d_my_ix = to_device(my_ix);
  // every other rank's boxes, unless the level is replicated: my rhs goes to
  // every peer (one packed copy, m_free_space.f90:152-153's allreduce)
  if (c->n_ranks > 1 && !(L && L->replicated)) {
    const int nc = c->bsl[fft_lvl];
    Transfer& T = S->gather;
    T.item_doubles = nc * nc * nc;
    std::vector<Rec> snd, rcv;
    for (int id : c->ids[fft_lvl]) {
      const int r = c->rank_of[id - 1];
      if (r == c->rank) {
        for (int q = 0; q < c->n_ranks; q++)
          if (q != c->rank) snd.push_back({q, (long long)id, c->local_index[id], 0});
      } else {
        rcv.push_back({r, (long long)id, id, 0});
      }
    }
    T.send = group(snd, 1);
    T.recv = group(rcv, 1);
    finalize_transfer(T);
    for (auto& p : T.send) p.offset = 0;   // the same packed boxes for every peer
    std::vector<int> rix;
    for (auto& p : T.recv)
      for (int id : p.items)
        for (int d = 0; d < 3; d++) rix.push_back(c->ix[(size_t)(id - 1) * 3 + d]);
    S->d_recv_ix = to_device(rix);
    dmalloc(&S->d_send, sizeof(double) * (size_t)S->n_my * T.item_doubles);
    dmalloc(&S->d_recv, sizeof(double) * (size_t)T.n_recv * T.item_doubles);
  }
  S->fft_lvl = fft_lvl;
}

// the interpolated Dirichlet values of phi on every physical face of every
// box here (ghost_cells_free_bc via mg_phi_bc_store, m_free_space.f90:174,
// 216-270) as phi's boundary table, then mg_phi_bc_store itself
void free_store_bc(omg_ctx* c, omg_free_state* S, const double* box_r_min) {
  const int k = 0;   // phi
  for (auto& kv : c->d_face_off_lvl[k]) dfree(kv.second);
  for (auto& kv : c->d_face_type_lvl[k]) dfree(kv.second);
  c->d_face_off_lvl[k].clear();
  c->d_face_type_lvl[k].clear();
  c->h_face_off_lvl[k].clear();
  c->h_face_type_lvl[k].clear();
  dfree(c->d_face_data[k]);
  std::vector<FreeFace> faces;
  long long n_data = 0;
  for (auto& kv : c->levels) {
    Level& L = kv.second;
    if (!L.n) continue;
    const std::vector<double>& dr = c->drl[kv.first];
    std::vector<long long> off(L.n * 6, -1);
    std::vector<int> typ(L.n * 6, 0);
    for (int b = 0; b < L.n; b++)
      for (int nb = 1; nb <= 6; nb++) {
        if (L.h_nbk[(size_t)b * 6 + nb - 1] != NB_PHYS) continue;
        const int id = L.ids[b];
        FreeFace f;
        for (int d = 0; d < 3; d++) {
          f.rmin[d] = box_r_min ? box_r_min[(size_t)(id - 1) * 3 + d]
                                : S->r_min[d] + (double)((c->ix[(size_t)(id - 1) * 3 + d] - 1) * L.nc) * dr[d];
          f.dr[d] = dr[d];
        }
        f.off = n_data;
        f.nb = nb;
        f.nc = L.nc;
        faces.push_back(f);
        off[(size_t)b * 6 + nb - 1] = n_data;
        typ[(size_t)b * 6 + nb - 1] = OMG_BC_DIRICHLET;
        n_data += (long long)L.nc * L.nc;
      }
    c->d_face_off_lvl[k][kv.first] = to_device(off);
    c->d_face_type_lvl[k][kv.first] = to_device(typ);
    c->h_face_off_lvl[k][kv.first] = off;
    c->h_face_type_lvl[k][kv.first] = typ;
  }
  for (int nb = 0; nb < 6; nb++) {
    c->bc[k].type[nb] = OMG_BC_DIRICHLET;
    c->bc[k].value[nb] = 0.0;
  }
  dmalloc(&c->d_face_data[k], sizeof(double) * std::max(n_data, 1LL));
  FreeFace* d_faces = to_device(faces);
  launch_free_bc_faces(d_faces, (int)faces.size(), S->d_planes, S->G, S->P, c->d_face_data[k], c->stream);
  phi_bc_store(c);   // synchronises the stream
  dfree(d_faces);
}

// mg_poisson_free_3d (m_free_space.f90:36-214)
double poisson_free_3d(omg_ctx* c, bool new_rhs, double max_fft_frac, bool fmgcycle, bool want_max_res,
                       const double* r_min, const double* box_r_min) {
  if (!c->free_state) c->free_state = new omg_free_state;
  omg_free_state* S = c->free_state;
  if (!S->initialized && !new_rhs)
    throw OmgError("mg_poisson_free_3d: first call requires new_rhs = .true.");
  if (c->op != OP_LPL) throw OmgError("mg_poisson_free_3d: laplacian operator required");
  // mg_number_of_unknowns (m_data_structures.f90:482-492)
  long long n_total = 0;
  for (int l = c->first_normal; l <= c->highest; l++) n_total += (long long)c->leaves[l].size();
  n_total *= (long long)c->box_size * c->box_size * c->box_size;
  // mg_highest_uniform_lvl (m_data_structures.f90:469-479)
  int lvl = c->first_normal;
  for (; lvl <= c->highest - 1; lvl++)
    if (!c->leaves[lvl].empty() && !c->parents[lvl].empty()) break;
  // the highest level small enough for the FFT solve (:83-90)
  for (; lvl >= c->lowest + 1; lvl--) {
    const long long n_lvl = (long long)c->ids[lvl].size() * c->box_size * c->box_size * c->box_size;
    if ((double)n_lvl <= max_fft_frac * (double)n_total) break;
  }
  const int fft_lvl = lvl;
  const bool new_grid = !S->initialized || S->fft_lvl != fft_lvl;
  // domain_size_lvl(:, fft_lvl) + 2 (:95)
  int nx[3] = {0, 0, 0};
  const int nc_f = c->bsl[fft_lvl];
  for (int id : c->ids[fft_lvl])
    for (int d = 0; d < 3; d++) nx[d] = std::max(nx[d], c->ix[(size_t)(id - 1) * 3 + d] * nc_f);
  for (int d = 0; d < 3; d++) nx[d] += 2;
  // the reference creates PSolver's kernel for (nx(1), nx(3), nx(3))
  // (m_free_space.f90:118-120) and solves on (nx(1), nx(2), nx(3)): the two
  // agree only when ny == nz, the only case it can solve (and that its
  // fixtures cover); anything else is refused rather than guessed
  if (nx[1] != nx[2])
    throw OmgError("mg_poisson_free_3d: the FFT level needs ny == nz (the reference's kernel is built for "
                   "(nx, nz, nz), m_free_space.f90:118-120)");
  const double h[3] = {c->drl[fft_lvl][0], c->drl[fft_lvl][1], c->drl[fft_lvl][2]};
  if (S->initialized && new_grid) free_grid_release(S);
  for (int d = 0; d < 3; d++) S->r_min[d] = r_min ? r_min[d] : 0.0;
  if (new_grid) {
    for (int l = c->highest; l >= fft_lvl + 1; l--) restrict_lvl(c, 2, l);   // :113-115
    free_new_grid(c, S, fft_lvl, nx, h);
    // interp_bc's plane geometry (:128-139): tangential dims of each face
    const int tdim[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    for (int d = 0; d < 3; d++)
      for (int q = 0; q < 2; q++) {
        S->P.inv_dr[d][q] = 1.0 / h[tdim[d][q]];
        S->P.r_min[d][q] = S->r_min[tdim[d][q]] - 0.5 * h[tdim[d][q]];
      }
  }
  if (new_rhs) {
    const FreeGrid& G = S->G;
    const double rhs_fac = -1.0 / (4.0 * std::acos(-1.0));   // :67
    Level* L = level_ptr(c, fft_lvl);
    const size_t nr = (size_t)G.N[0] * G.N[1] * G.N[2], nz = (size_t)(G.N[0] / 2 + 1) * G.N[1] * G.N[2];
    {
      Prof p(c, "free_fft_solve", (double)nr, fft_lvl);
      HIPCHK(hipMemsetAsync(S->d_R, 0, sizeof(double) * nr, c->stream));
      if (L) launch_free_gather(L->view(), S->d_my, S->d_my_ix, S->n_my, G, rhs_fac, S->d_R, c->stream);
      Transfer& T = S->gather;
      if (T.n_send || T.n_recv) {
        if (L) launch_free_pack(L->view(), S->d_my, S->n_my, S->d_send, c->stream);
        exchange(c, T, S->d_send, S->d_recv);
        launch_free_scatter(S->d_recv, S->d_recv_ix, T.n_recv, nc_f, G, rhs_fac, S->d_R, c->stream);
      }
      FFTCHK(hipfftExecD2Z(S->fwd, S->d_R, (hipfftDoubleComplex*)S->d_Z));
      launch_free_mul(S->d_Z, S->d_karray, (long long)nz, c->stream);
      FFTCHK(hipfftExecZ2D(S->inv, (hipfftDoubleComplex*)S->d_Z, S->d_R));
      launch_free_planes(S->d_R, G, S->d_planes, c->stream);
    }
    free_store_bc(c, S, box_r_min);
    // the solution as the initial guess on the FFT level, incl. ghosts (:176-183)
    if (L) launch_free_guess(L->view(), S->d_my, S->d_my_ix, S->n_my, G, S->d_R, c->stream);
    phi_dirty(c, fft_lvl);
    for (int l = fft_lvl; l >= c->lowest + 1; l--) restrict_lvl(c, 1, l);   // :186-188
    for (int l = fft_lvl; l <= c->highest - 1; l++) {                        // :191-195
      prolong(c, l, 1, 1, 0);
      fill_gc_lvl(c, l + 1, 1);
    }
    S->initialized = true;
  }
  if (fft_lvl < c->highest)   // :201-208
    return run_cycle(c, 16 + (want_max_res ? 2 : 0) + (fmgcycle ? 1 : 0), [&] {
      return fmgcycle ? fas_fmg(c, true, want_max_res) : fas_vcycle(c, c->lowest - 1, want_max_res, true);
    });
  return 0.0;
}

// ---------------------------------------------------------------------------
// Plan builder (device side of mg_allocate_storage, m_allocate_storage.f90:51-99,
// and of the three buffer dry runs m_ghost_cells.f90:17-62, m_restrict.f90:
// 16-69, m_prolong.f90:16-48).
void free_levels(omg_ctx* c) {
  free_state_destroy(c);   // the FFT level belongs to the old tree
  for (auto& kv : c->levels) {
    Level& L = kv.second;
    dfree(L.d_data); L.d_phi = nullptr; dfree(L.d_nbk); dfree(L.d_nba); dfree(L.d_sendpos); dfree(L.d_rb);
    dfree(L.d_topo);
    rbh_free(L);
    dfree(L.d_parents); dfree(L.d_leaves); dfree(L.d_parent_local); dfree(L.d_dix); dfree(L.d_parmask);
    dfree(L.d_rbgv);
    dfree(L.d_pairs); dfree(L.d_sendbuf); dfree(L.d_recvbuf); dfree(L.d_scratch); dfree(L.d_scratch_rhs);
    dfree(L.d_rhs_lex);
    dfree(L.d_xlay);
    dfree(L.d_galt);
    dfree(L.d_phi_buf); dfree(L.d_b3); dfree(L.d_b3c); L.n_b3 = 0; L.h_b3.clear();
    dfree(L.d_physbox);
    dfree(L.d_rbsend); dfree(L.d_rbrecv); dfree(L.d_bnd); dfree(L.d_int); dfree(L.d_push0); dfree(L.d_bndface);
    for (Transfer* T : {&L.halo, &L.restr, &L.prol, &L.rbx, &L.repl, &L.deep_phi, &L.deep_rhs}) {
      dfree(T->d_send_items);
      dfree(T->d_recv_items);
    }
  }
  c->levels.clear();
  for (int iv = 0; iv < kMaxVars; iv++) {
    for (auto& kv : c->d_face_off_lvl[iv]) dfree(kv.second);
    for (auto& kv : c->d_face_type_lvl[iv]) dfree(kv.second);
    c->d_face_off_lvl[iv].clear();
    c->d_face_type_lvl[iv].clear();
    c->h_face_off_lvl[iv].clear();
    c->h_face_type_lvl[iv].clear();
    dfree(c->d_face_data[iv]);
  }
}

// whether k_gsrb3's 32-bit byte offsets reach every box of a variable
bool block3_addressable(long long n_boxes, long long stride) {
  return (unsigned long long)n_boxes * (unsigned long long)stride * 8ull <= 0xFFFFFFFFull;
}

// boxes per column in z: 16 on levels of >= 32768 boxes, 4 down to 4096, below
// that (levels that take the passes with OMG_BLOCK3_MIN_BOXES lowered) 2, for
// more workgroups (OMG_BLOCK3_SMALL_COL); OMG_BLOCK3_COLUMN: all levels
int b3_column(const omg_ctx* c, int n) {
  if (c->b3_col) return c->b3_col;
  return n / (kB3TX * 8) >= 2048 ? 16 : (n >= kB3MinBoxes ? 4 : c->b3_col_small);
}

// k_gsrb3's columns (launch_gsrb3): a level of at least kB3MinBoxes boxes of
// 16^3 whose faces are all same-GPU boxes of the level or physical (a uniform
// level on one GPU) is tiled by columns of kB3TX boxes in x and up to kB3MaxZ
// in z, each with the boxes around it; the level then gets phi's second
// buffer.  Columns are ordered by z block, then Morton order in x / y, so that
// each XCD's run of workgroups (xcd_box) is one compact patch whose halo
// columns its own L2 holds.  A physical face (round 6) is a flag of the
// column (kB3LenMask), the same for all its boxes, and the slot across it names
// the box whose face it is.  Any face or tiling that does not fit: no records.
void build_block3(omg_ctx* c, Level& L) {
  if (g_host_only || c->host_only || L.nc != 16 || L.n < c->b3_min_boxes || L.replicated || L.deep) return;
  // k_gsrb3 / k_gsrb4 address a variable with 32-bit byte offsets
  // (omg_block.hip b3_ld / b3_st): 95,325 boxes of 16^3 at most
  if (!block3_addressable(L.n + L.n_prox, L.stride)) return;
  for (int8_t k : L.h_nbk)
    if (k != NB_LOCAL && !(k == NB_PHYS && !c->no_block3_phys)) return;
  const int n = L.n;
  // face f: 0 x-, 1 x+, 2 y-, 3 y+, 4 z-, 5 z+; across a physical face the box itself
  auto phys = [&](int b, int f) { return L.h_nbk[(size_t)b * 6 + f] == NB_PHYS; };
  auto nb = [&](int b, int f) { return phys(b, f) ? b : L.h_nba[(size_t)b * 6 + f]; };
  auto ixd = [&](int b, int d) { return c->ix[(size_t)(L.ids[b] - 1) * 3 + d] - 1; };
  auto spread = [](unsigned v) {
    unsigned long long r = 0;
    for (int q = 0; q < 20; q++) r |= (unsigned long long)((v >> q) & 1u) << (2 * q);
    return r;
  };
  std::vector<std::pair<unsigned long long, std::vector<int>>> cols;
  std::vector<int> covered(n, 0);
  bool any_phys = false;
  // columns of 16 boxes on levels of >= 32768 boxes, else 4: C3's level 1
  // 857 / 759 us per pass against 875 / 772 with 8 (1024 workgroups, fewer
  // halo planes per box; profiles/r05/s40_block3_z16_ab.txt) and 898 / 789
  // with 4 (s38); on its 4096-box level 8 gained nothing, and two-box columns,
  // twice the workgroups, took 110 us a pass against 102
  const int nzb = b3_column(c, L.n);
  static_assert(kB3MaxZ >= 16, "column records hold 16 boxes");
  for (int h = 0; h < n; h++) {
    if (ixd(h, 0) % kB3TX || ixd(h, 2) % nzb) continue;
    std::vector<int> zc{h};
    while ((int)zc.size() < nzb && !phys(zc.back(), 5)) {
      const int up = nb(zc.back(), 5);
      if (ixd(up, 2) % nzb == 0) break;   // the next column's first box
      zc.push_back(up);
    }
    const int len = (int)zc.size();
    // the column's physical faces: x-, x+, y-, y+ alike for all its boxes (and
    // none between the tile's boxes), z- of its first box, z+ of its last
    int fl = (phys(zc[0], 4) ? 16 : 0) | (phys(zc[len - 1], 5) ? 32 : 0);
    for (int z = 0; z < len; z++) {
      int t[kB3TX];
      t[0] = zc[z];
      for (int xs = 1; xs < kB3TX; xs++) {
        if (phys(t[xs - 1], 1)) return;
        t[xs] = nb(t[xs - 1], 1);
      }
      int f = (phys(t[0], 0) ? 1 : 0) | (phys(t[kB3TX - 1], 1) ? 2 : 0);
      for (int xs = 0; xs < kB3TX; xs++) {
        const int fy = (phys(t[xs], 2) ? 4 : 0) | (phys(t[xs], 3) ? 8 : 0);
        if (xs && fy != (f & 12)) return;
        f |= fy;
      }
      if (z && f != (fl & 15)) return;
      fl |= f;
    }
    any_phys |= fl != 0;
    std::vector<int> r(kB3Rec, 0);
    r[0] = len | fl << 8;
    for (int zs = 0; zs <= len + 1; zs++) {
      const int cb = zs == 0 ? nb(zc[0], 4) : (zs == len + 1 ? nb(zc[len - 1], 5) : zc[zs - 1]);
      int* row = &r[1 + kB3S * zs];
      // the tile's row of boxes along x, then the rows below and above it in
      // y; a grid: the rows' x neighbours agree with the y neighbours' chain
      // (except where a slot stands across a physical face)
      row[kB3TX + 2] = nb(cb, 0);
      for (int xs = 1; xs <= kB3TX + 1; xs++) row[(kB3TX + 2) + xs] = xs == 1 ? cb : nb(row[(kB3TX + 2) + xs - 1], 1);
      for (int xs = 0; xs < kB3TX + 2; xs++) {
        const int mid = row[(kB3TX + 2) + xs];
        row[xs] = nb(mid, 2);
        row[2 * (kB3TX + 2) + xs] = nb(mid, 3);
        if (zs >= 1 && zs <= len && xs >= 1 && xs <= kB3TX) covered[mid]++;
      }
      for (int ys = 0; ys < 3; ys += 2)
        for (int xs = (fl & 1) ? 1 : 0; xs + 1 < kB3TX + ((fl & 2) ? 1 : 2); xs++)
          if (nb(row[(kB3TX + 2) * ys + xs], 1) != row[(kB3TX + 2) * ys + xs + 1]) return;
    }
    const unsigned long long key = ((unsigned long long)(ixd(h, 2) / nzb) << 40) |
                                   (spread((unsigned)(ixd(h, 0) / kB3TX)) | (spread((unsigned)ixd(h, 1)) << 1));
    cols.emplace_back(key, std::move(r));
  }
  for (int b = 0; b < n; b++)
    if (covered[b] != 1) return;
  std::sort(cols.begin(), cols.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<int> flat;
  flat.reserve(cols.size() * kB3Rec);
  for (auto& cr : cols) flat.insert(flat.end(), cr.second.begin(), cr.second.end());
  L.n_b3 = (int)cols.size();
  L.b3_phys = any_phys;
  L.d_b3 = to_device(flat);
  L.h_b3 = std::move(flat);
  dmalloc(&L.d_phi_buf, sizeof(double) * (size_t)L.n * L.stride, true);
}

// The ghost terms of the block passes' physical faces: bc_to_gc's c0 * b, c1,
// c2 per face (m_ghost_cells.f90:665-766; k_gsrb_tile's phys_ghost, the same
// expressions), for constant boundary values only; false when the level's
// are tabulated (a boundary callback) or stored with phi.
bool b3_phys_args(omg_ctx* c, int lvl, const Level& L, B3Phys& P) {
  if (c->phi_bc_data_stored) return false;
  auto it = c->d_face_off_lvl[0].find(lvl);
  if (it != c->d_face_off_lvl[0].end() && it->second) return false;
  for (int nb = 1; nb <= 6; nb++) {
    const int type = c->bc[0].type[nb - 1];
    const double bv = c->bc[0].value[nb - 1];
    double c0, c1, c2;
    if (type == OMG_BC_DIRICHLET) {
      c0 = 2; c1 = -1; c2 = 0;
    } else if (type == OMG_BC_NEUMANN) {
      c0 = L.dr[(nb - 1) >> 1] * ((nb & 1) ? -1.0 : 1.0); c1 = 1; c2 = 0;
    } else {
      c0 = 0; c1 = 2; c2 = -1;
    }
    P.k[nb - 1] = c0 * bv;
    P.c1[nb - 1] = c1;
    P.c2[nb - 1] = c2;
  }
  return true;
}

// whether a block pass (k_gsrb3 / k_gsrb4) may smooth the level now: records,
// consistent ghosts, an operator it has; ph: its physical faces' terms (null:
// none), P their storage
bool b3_usable(omg_ctx* c, int lvl, B3Phys& P, const B3Phys*& ph) {
  const Level* L = level_ptr(c, lvl);
  ph = nullptr;
  if (!L || !L->d_b3 || !(L->phi_gc_ok || (L->gc_deferred && !L->b3_phys)) || !gsrb3_op_ok(c->op) ||
      c->no_block3)
    return false;
  if (L->b3_phys) {
    if (!b3_phys_args(c, lvl, *L, P)) return false;
    ph = &P;
  }
  return true;
}

// k_gsrb3's correct_children form (launch_gsrb3's ccols) for the columns of F:
// every column of an even number of boxes starts at a coarse box's corner in x
// and z, its fine boxes are the children of its coarse boxes, and every coarse
// box is the own box of exactly two columns (its two halves in y), on a
// coarse level of 16^3 boxes whose faces are all same-GPU boxes.
void build_block3c(omg_ctx* c, Level& F, const Level& C) {
  if (F.h_b3.empty() || C.nc != 16 || C.replicated || C.n == 0 || F.n != 8 * C.n || F.deep != C.deep) return;
  if (!block3_addressable(C.n + C.n_prox, C.stride)) return;
  if (!F.deep)
    for (int8_t k : C.h_nbk)
      if (k != NB_LOCAL) return;
  for (int b = 0; b < F.n; b++)
    if (F.parent_local[b] < 0) return;
  // the coarse boxes by their neighbours: C's own table on one GPU; on a
  // split level (deep halo on both levels) the global tree, a box on another
  // rank standing for its proxy in C's arena (deep_res fills its res)
  Tree T{c};
  auto cslot = [&](int id) {
    if (id > 0 && T.rank(id) == c->rank) return c->local_index[id];
    auto it = std::lower_bound(C.prox_ids.begin(), C.prox_ids.end(), id);
    return it != C.prox_ids.end() && *it == id ? C.n + (int)(it - C.prox_ids.begin()) : -1;
  };
  auto cid = [&](int x) { return x < C.n ? C.ids[x] : C.prox_ids[x - C.n]; };
  auto nbc = [&](int b, int f) {
    if (!F.deep) return C.h_nba[(size_t)b * 6 + f];
    const int id = T.nbr(cid(b), f + 1);
    return id > 0 ? cslot(id) : -1;
  };
  auto dix = [&](int b, int q) { return (F.dix_packed[b] >> (10 * q)) & 1023; };
  std::vector<int> out((size_t)F.n_b3 * kB3CRec, 0);
  std::vector<int> own(C.n, 0);
  for (int q = 0; q < F.n_b3; q++) {
    const int* r = &F.h_b3[(size_t)q * kB3Rec];
    if (r[0] > kB3LenMask) return;   // (physical faces: the plain passes only)
    const int len = r[0], lenc = len / 2;
    if (len % 2) return;
    auto fine = [&](int zs, int xs) { return r[1 + kB3S * zs + (kB3TX + 2) + xs]; };
    const int b0 = fine(1, 1);
    if (dix(b0, 0) != 0 || dix(b0, 2) != 0) return;
    int* o = &out[(size_t)q * kB3CRec];
    o[0] = dix(b0, 1);
    int zc[kB3MaxZ / 2 + 2];
    zc[1] = F.parent_local[b0];
    for (int z = 2; z <= lenc; z++) zc[z] = nbc(zc[z - 1], 5);
    if (F.deep)
      for (int z = 2; z <= lenc; z++)
        if (zc[z] < 0 || zc[z] >= C.n) return;   // (a column's coarse boxes are this rank's)
    zc[0] = nbc(zc[1], 4);
    zc[lenc + 1] = nbc(zc[lenc], 5);
    for (int z = 0; z <= lenc + 1; z++) {
      int* row = o + 1 + 9 * z;
      row[4] = zc[z];
      row[3] = nbc(zc[z], 0);
      row[5] = nbc(zc[z], 1);
      for (int xs = 0; xs < 3; xs++) {
        row[xs] = nbc(row[3 + xs], 2);
        row[6 + xs] = nbc(row[3 + xs], 3);
      }
      for (int q2 = 0; q2 < 9; q2++)
        if (row[q2] < 0) return;
      for (int ys = 0; ys < 3; ys += 2)
        for (int xs = 0; xs < 2; xs++)
          if (nbc(row[3 * ys + xs], 1) != row[3 * ys + xs + 1]) return;
      if (z >= 1 && z <= lenc) own[zc[z]]++;
    }
    for (int zs = 1; zs <= len; zs++)
      for (int xs = 1; xs <= kB3TX; xs++) {
        const int fb = fine(zs, xs);
        if (F.parent_local[fb] != zc[(zs + 1) / 2] || dix(fb, 0) != (xs - 1) * 8 || dix(fb, 1) != o[0] ||
            dix(fb, 2) != ((zs - 1) & 1) * 8)
          return;
      }
  }
  for (int b = 0; b < C.n; b++)
    if (own[b] != 2) return;
  F.d_b3c = to_device(out);
}

// ---------------------------------------------------------------------------
// Deep halo: k_gsrb3 / k_gsrb4 on a level split over GPUs.
// The reference fills the ghost layer after every substep
// (m_multigrid.f90:404-424, mg_fill_ghost_cells_lvl, m_ghost_cells.f90:131-175,
// whose remote part is one sort_and_transfer_buffers round,
// m_communication.f90:37-66).  A multi-substep pass instead reads the
// neighbours' cells up to 4 deep, so on a split level the remote boxes its
// columns read become proxy boxes of this rank (after its own boxes, in every
// variable), filled once per pass: phi of the colour the pass reads, rhs when
// it changed.  The pass then runs exactly as on one GPU; its store wave's
// pushes into proxies are dropped, and the remote faces' ghosts of this rank's
// boxes arrive by the level's halo plan after it.
//
// What travels: a proxy B is read by the columns of this rank's boxes A in
// its 26-neighbourhood; per dimension, B lies below A (its top 4 layers are
// read), above (its bottom 4) or level with A (all 16): a product of ranges,
// whose union over those A is sent as 4^3-cell bricks (launch_deep_copy).  Every rank derives the same regions from the global
// tree, so the brick lists pair up key for key (key 64*id + brick).
//
// Where: 16^3 levels, every face a box of the level (uniform, periodic or
// interior), x pairs of boxes (even ix and its x+ neighbour) on one rank, at
// least b3_min_boxes boxes on every rank holding some, and byte offsets of
// every rank's boxes + proxies under 4 GiB; decided alike on every rank.  On
// a level of leaves rhs changes only by the periodic mean, which the proxies
// follow; a level with parents gets its rhs from update_coarse every cycle,
// so its proxies' rhs travels once per cycle.  Such a level (C3's level 0 at
// N > 1) also stores res for the correction form above it (the RES pass), and
// its proxies get that res too (deep_res).
// the box at offset o (components -1..1) from id, walking x, y, z in turn
// (zyx: the reverse order); 0 when the walk leaves the level's boxes
int deep_walk(const Tree& T, int id, const int o[3], bool zyx = false) {
  for (int s = 0; s < 3; s++) {
    const int d = zyx ? 2 - s : s;
    if (!o[d]) continue;
    id = T.nbr(id, 2 * d + (o[d] > 0 ? 2 : 1));
    if (id <= 0) return 0;
  }
  return id;
}

template <typename F>
void deep_offsets(F&& f) {
  for (int z = -1; z <= 1; z++)
    for (int y = -1; y <= 1; y++)
      for (int x = -1; x <= 1; x++)
        if (x || y || z) {
          const int o[3] = {x, y, z};
          f(o);
        }
}

// the bricks box B shows a box A at offset o from B (A reads B's 4 layers
// toward it, all 16 across): bit bx + 4 by + 16 bz
unsigned long long deep_bricks(const int o[3]) {
  unsigned long long m = 0;
  for (int bz = 0; bz < 4; bz++)
    for (int by = 0; by < 4; by++)
      for (int bx = 0; bx < 4; bx++) {
        const int b[3] = {bx, by, bz};
        bool in = true;
        for (int d = 0; d < 3; d++) in &= o[d] == 0 || b[d] == (o[d] > 0 ? 3 : 0);
        if (in) m |= 1ull << (bx + 4 * by + 16 * bz);
      }
  return m;
}

// (before the level's arena is allocated: sets n_prox, which sizes it)
void plan_deep(omg_ctx* c, Level& L) {
  const int l = L.lvl, me = c->rank;
  L.deep = false;
  L.n_prox = 0;
  L.prox_ids.clear();
  if (c->n_ranks == 1 || L.replicated || L.nc != 16 || c->no_block3 || c->no_deep) return;
  Tree T{c};
  const auto& ids = c->ids[l];
  if (ids.empty()) return;
  std::map<int, std::vector<int>> by_rank;
  bool split = false;
  for (int id : ids) {
    by_rank[T.rank(id)].push_back(id);
    for (int nb = 1; nb <= 6; nb++) {
      const int nid = T.nbr(id, nb);
      if (nid <= 0 || T.lvl(nid) != l) return;   // physical or refinement-boundary face
      split |= T.rank(nid) != T.rank(id);
    }
  }
  if (!split) return;
  auto ixd = [&](int id, int d) { return c->ix[(size_t)(id - 1) * 3 + d] - 1; };
  for (int id : ids) {
    const int odd = ixd(id, 0) & 1, pr = T.nbr(id, odd ? 1 : 2);
    if (T.rank(pr) != T.rank(id) || T.nbr(pr, odd ? 2 : 1) != id || (ixd(pr, 0) & 1) == odd) return;
    bool grid = true;
    deep_offsets([&](const int* o) { grid &= deep_walk(T, id, o) == deep_walk(T, id, o, true); });
    if (!grid) return;
  }
  // every rank: enough boxes, and its boxes + proxies addressable by k_gsrb3's
  // 32-bit byte offsets
  std::vector<int> stamp((size_t)c->n_boxes + 1, -1);
  const unsigned long long box_bytes = 8ull * (unsigned long long)(((stored_cells(16) + 63) / 64) * 64);
  for (auto& kv : by_rank) {
    if ((int)kv.second.size() < c->b3_min_boxes) return;
    long long np = 0;
    for (int id : kv.second)
      deep_offsets([&](const int* o) {
        const int b = deep_walk(T, id, o);
        if (T.rank(b) != kv.first && stamp[b] != kv.first) {
          stamp[b] = kv.first;
          np++;
        }
      });
    if ((unsigned long long)(kv.second.size() + np) * box_bytes > 0xFFFFFFFFull) return;
  }
  L.deep = true;
  // proxies (this rank reads them) and what the peers read of this rank's boxes
  // (box B at offset o from my box A: A reads B's bricks at -o from B; and
  // the peer's box B reads my A's bricks at o from A)
  std::map<int, unsigned long long> need;
  std::map<std::pair<int, int>, unsigned long long> give;
  for (int id : L.ids) {
    if (T.rank(id) != me) continue;
    deep_offsets([&](const int* o) {
      const int b = deep_walk(T, id, o), q = T.rank(b);
      if (q == me) return;
      const int mo[3] = {-o[0], -o[1], -o[2]};
      need[b] |= deep_bricks(mo);
      give[{q, id}] |= deep_bricks(o);
    });
  }
  std::map<int, int> pidx;
  for (auto& kv : need) {
    pidx[kv.first] = L.n + (int)L.prox_ids.size();
    L.prox_ids.push_back(kv.first);
  }
  L.n_prox = (int)L.prox_ids.size();
  std::vector<Rec> rs, rr;
  for (auto& kv : need)
    for (int br = 0; br < 64; br++)
      if ((kv.second >> br) & 1) rr.push_back({T.rank(kv.first), 64LL * kv.first + br, pidx[kv.first], br});
  for (auto& kv : give)
    for (int br = 0; br < 64; br++)
      if ((kv.second >> br) & 1)
        rs.push_back({kv.first.first, 64LL * kv.first.second + br, c->local_index[kv.first.second], br});
  for (Transfer* X : {&L.deep_phi, &L.deep_rhs}) {
    X->send = group(rs, 2);
    X->recv = group(rr, 2);
    X->send_ints = X->recv_ints = 2;
    X->item_doubles = X == &L.deep_phi ? 32 : 64;
    finalize_transfer(*X);
  }
  L.prox_rhs_ok = false;
  // the columns (build_block3's, over global ids: a column's boxes are this
  // rank's, the boxes around it this rank's or proxies)
  auto mine = [&](int id) { return id > 0 && T.rank(id) == me; };
  auto slot = [&](int id) {
    if (mine(id)) return c->local_index[id];
    auto it = pidx.find(id);
    if (it == pidx.end()) throw OmgError("plan_deep: a column reads a box outside the proxies");
    return it->second;
  };
  const int nzb = b3_column(c, L.n);
  std::vector<std::pair<unsigned long long, std::vector<int>>> cols;
  std::vector<int> covered(L.n, 0);
  auto spread = [](unsigned v) {
    unsigned long long r = 0;
    for (int q = 0; q < 20; q++) r |= (unsigned long long)((v >> q) & 1u) << (2 * q);
    return r;
  };
  for (int h : L.ids) {
    if (!mine(h) || ixd(h, 0) % kB3TX || !(ixd(h, 2) % nzb == 0 || !mine(T.nbr(h, 5)))) continue;
    std::vector<int> zc{h};
    while ((int)zc.size() < nzb) {
      const int up = T.nbr(zc.back(), 6);
      if (!mine(up) || ixd(up, 2) % nzb == 0) break;
      zc.push_back(up);
    }
    const int len = (int)zc.size();
    std::vector<int> r(kB3Rec, 0);
    r[0] = len;
    for (int zs = 0; zs <= len + 1; zs++) {
      const int cb = zs == 0 ? T.nbr(zc[0], 5) : (zs == len + 1 ? T.nbr(zc[len - 1], 6) : zc[zs - 1]);
      int g[3][kB3TX + 2];
      g[1][0] = T.nbr(cb, 1);
      for (int xs = 1; xs <= kB3TX + 1; xs++) g[1][xs] = xs == 1 ? cb : T.nbr(g[1][xs - 1], 2);
      for (int xs = 0; xs < kB3TX + 2; xs++) {
        g[0][xs] = T.nbr(g[1][xs], 3);
        g[2][xs] = T.nbr(g[1][xs], 4);
      }
      for (int ys = 0; ys < 3; ys++)
        for (int xs = 0; xs < kB3TX + 2; xs++) {
          if (zs >= 1 && zs <= len && ys == 1 && xs >= 1 && xs <= kB3TX) {
            if (!mine(g[ys][xs])) throw OmgError("plan_deep: a column box on another rank");
            covered[c->local_index[g[ys][xs]]]++;
          }
          r[1 + kB3S * zs + (kB3TX + 2) * ys + xs] = slot(g[ys][xs]);
        }
    }
    const unsigned long long key = ((unsigned long long)(ixd(h, 2) / nzb) << 40) |
                                   (spread((unsigned)(ixd(h, 0) / kB3TX)) | (spread((unsigned)ixd(h, 1)) << 1));
    cols.emplace_back(key, std::move(r));
  }
  for (int b = 0; b < L.n; b++)
    if (covered[b] != 1) throw OmgError("plan_deep: the columns do not cover the level once");
  std::sort(cols.begin(), cols.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  std::vector<int> flat;
  flat.reserve(cols.size() * kB3Rec);
  for (auto& cr : cols) flat.insert(flat.end(), cr.second.begin(), cr.second.end());
  L.n_b3 = (int)cols.size();
  L.d_b3 = to_device(flat);
  L.h_b3 = std::move(flat);
}

void build_plan(omg_ctx* c) {
  Tree T{c};
  const int me = c->rank;
  c->local_index.assign(c->n_boxes + 1, -1);
  // Replicated coarse levels: the lowest levels, while they hold at most
  // rep_cells cells and neither leaves nor refinement boundaries, live on every
  // rank.  Their exchanges (latency-bound at a few boxes per GPU) disappear:
  // the restriction into the highest replicated level goes to every rank, and
  // the prolongation out of it is local everywhere.  Bits do not change: each
  // box's arithmetic is the same wherever it runs, and get_sum reads leaves only.
  c->rep_lvl = INT_MIN;
  if (c->rep_cells > 0 && c->n_ranks > 1)
    for (int l = c->lowest; l < c->highest; l++) {
      const long long nc = c->bsl[l];
      if ((long long)c->ids[l].size() * nc * nc * nc > c->rep_cells || !c->leaves[l].empty() ||
          !c->ref_bnds[l].empty())
        break;
      c->rep_lvl = l;
    }
  auto owns = [&](int id) { return T.lvl(id) <= c->rep_lvl || T.rank(id) == me; };
  for (int l = c->lowest; l <= c->highest; l++) {
    Level& L = c->levels[l];
    L.lvl = l;
    L.nc = c->bsl[l];
    L.replicated = l <= c->rep_lvl;
    for (int d = 0; d < 3; d++) L.dr[d] = c->drl[l][d];
    for (int id : c->ids[l])
      if (owns(id)) {
        c->local_index[id] = (int)L.ids.size();
        if (T.rank(id) == me) L.host_local.push_back((int)L.ids.size());
        L.ids.push_back(id);
      }
    L.n = (int)L.ids.size();
    L.stride = ((stored_cells(L.nc) + 63) / 64) * 64;   // 512-B aligned boxes
    if (L.replicated) {
      // the host's boxes of this level go to every peer (upload_level)
      std::vector<Rec> rs, rr;
      for (int b = 0; b < L.n; b++) {
        const int id = L.ids[b];
        if (T.rank(id) == me) {
          for (int r = 0; r < c->n_ranks; r++)
            if (r != me) rs.push_back({r, (long long)id, b, 0});
        } else {
          rr.push_back({T.rank(id), (long long)id, b, 0});
        }
      }
      L.repl.send = group(rs, 1);
      L.repl.recv = group(rr, 1);
      L.repl.item_doubles = (int)L.stride;
      finalize_transfer(L.repl);
    }
  }
  for (int l = c->lowest; l <= c->highest; l++) {
    Level& L = c->levels[l];
    const int nc = L.nc;
    // deep halo on a split level (k_gsrb3 / k_gsrb4 there): the proxies
    // extend every variable of the arena
    plan_deep(c, L);
    // arena
    if (L.n) {
      const size_t bytes = sizeof(double) * (size_t)c->n_vars * (L.n + L.n_prox) * L.stride;
      dmalloc(&L.d_data, bytes, true);
      L.d_phi = L.d_data;
      if (L.deep && L.n_b3) dmalloc(&L.d_phi_buf, sizeof(double) * (size_t)(L.n + L.n_prox) * L.stride, true);
      if (c->debug && !g_host_only) {   // (L.view() needs only the arena fields here)
        launch_poison_ghosts(L.view(), c->n_vars, snan_value(), nullptr);
        HIPCHK(hipDeviceSynchronize());
      }
    }
    // neighbour table + halo receive plan
    L.h_nbk.assign((size_t)L.n * 6, NB_LOCAL);
    L.h_nba.assign((size_t)L.n * 6, 0);
    std::vector<Rec> hrecv, hsend, rbrecv, rbsend;
    for (int b = 0; b < L.n; b++) {
      const int id = L.ids[b];
      for (int nb = 1; nb <= 6; nb++) {
        const int nid = T.nbr(id, nb);
        const size_t f = (size_t)b * 6 + nb - 1;
        if (nid > 0) {
          if (owns(nid)) {
            L.h_nbk[f] = NB_LOCAL;
            L.h_nba[f] = c->local_index[nid];
          } else {
            L.h_nbk[f] = NB_REMOTE;
            hrecv.push_back({T.rank(nid), (long long)id * 6 + nb, (int)f, 0});
            // the neighbour sends the face of its own box toward us; we send ours
            hsend.push_back({T.rank(nid), (long long)nid * 6 + kNeighbRev[nb - 1], (int)f, 0});
          }
        } else if (nid == 0) {
          // refinement boundary: parent's neighbour at lvl-1 (fill_refinement_bnd :287-328)
          const int p_id = T.parent(id);
          const int p_nb = p_id > 0 ? T.nbr(p_id, nb) : 0;
          if (p_nb <= 0) throw OmgError("refinement boundary without coarse neighbour");
          if (!owns(p_nb)) {
            L.h_nbk[f] = NB_RBREM;
            rbrecv.push_back({T.rank(p_nb), (long long)id * 6 + nb, (int)f, 0});
            continue;
          }
          RBRec r;
          r.coarse_idx = c->local_index[p_nb];
          T.child_offset(id, r.dix);
          L.h_nbk[f] = NB_RB;
          L.h_nba[f] = (int)L.h_rb.size();
          L.h_rb.push_back(r);
        } else {
          L.h_nbk[f] = NB_PHYS;
          L.h_nba[f] = nid;
        }
      }
    }
    // coarse side of the refinement boundaries toward other ranks: my
    // ref_bnds at lvl-1 next to a refined box with children elsewhere
    // (buffer_refinement_boundaries, m_ghost_cells.f90:200-229)
    // (a replicated coarse level is on every rank: nothing to send)
    if (l > c->lowest && l - 1 > c->rep_lvl)
      for (int cid : c->ref_bnds[l - 1]) {
        if (T.rank(cid) != me) continue;
        for (int nb = 1; nb <= 6; nb++) {
          const int nid = T.nbr(cid, nb);
          if (nid <= 0 || T.child(nid, 1) <= 0) continue;
          const int rev = kNeighbRev[nb - 1];
          for (int s = 1; s <= 8; s++) {
            const int ch = T.child(nid, s);
            // children of nid on the face toward cid: child offset along the
            // normal matches the low/high side rev points to
            const int d = (nb + 1) >> 1, bit = ((s - 1) >> (d - 1)) & 1;
            if (bit != ((rev & 1) ? 0 : 1)) continue;
            if (ch <= 0 || T.rank(ch) == me) continue;
            int dd[3];
            T.child_offset(ch, dd);
            rbsend.push_back({T.rank(ch), (long long)ch * 6 + rev, c->local_index[cid], nb, pack_dix(dd)});
          }
        }
      }
    L.rbx.recv = group(rbrecv, 1);
    L.rbx.send = group(rbsend, 3);
    L.rbx.send_ints = 3;
    L.rbx.recv_ints = 1;
    L.rbx.item_doubles = nc * nc;
    finalize_transfer(L.rbx);
    L.halo.recv = group(hrecv, 1);
    L.halo.send = group(hsend, 1);
    L.halo.send_ints = L.halo.recv_ints = 1;
    L.halo.item_doubles = nc * nc;
    // receive slot of every remote face = its position in the receive buffer;
    // send slot = its position in the send buffer (wire order of each peer)
    std::vector<int> sendpos((size_t)L.n * 6, -1);
    {
      int pos = 0;
      for (auto& p : L.halo.recv)
        for (int f : p.items) L.h_nba[f] = pos++;
      pos = 0;
      for (auto& p : L.halo.send)
        for (int f : p.items) sendpos[f] = pos++;
    }
    finalize_transfer(L.halo);
    L.has_rb = !L.h_rb.empty() || L.rbx.n_recv > 0;
    L.has_remote = L.halo.n_send || L.halo.n_recv;
    L.has_phys = std::any_of(L.h_nbk.begin(), L.h_nbk.end(), [](int8_t k) { return k == NB_PHYS; });
    // (tiled box sizes: the red-black smoother's coarse-part buffer, for the
    // faces whose coarse box is on this GPU)
    if (!L.h_rb.empty() && !c->host_only && !c->no_rbgv &&
        (L.nc == 16 || L.nc == 8 || L.nc == 4 || L.nc == 2))
      dmalloc(&L.d_rbgv, sizeof(double) * L.n * 6 * L.nc * L.nc);
    L.rbgv_ok = false;
    {
      std::vector<int> pb;
      for (int b = 0; b < L.n; b++)
        for (int nb = 0; nb < 6; nb++)
          if (L.h_nbk[(size_t)b * 6 + nb] == NB_PHYS) {
            pb.push_back(b);
            break;
          }
      L.n_physbox = (int)pb.size();
      L.d_physbox = to_device(pb);
    }
    L.any_rb = L.any_phys = L.any_rbx = false;
    for (int id : c->ids[l])
      for (int nb = 1; nb <= 6; nb++) {
        const int nid = T.nbr(id, nb);
        L.any_rb |= nid == 0;
        L.any_phys |= nid < 0;
        if (nid == 0) {   // the coarse box across: the parent's neighbour
          const int p_id = c->parent[id - 1];
          const int p_nb = p_id > 0 ? T.nbr(p_id, nb) : 0;
          L.any_rbx |= p_nb > 0 && !(l - 1 <= c->rep_lvl) && c->rank_of[p_nb - 1] != c->rank_of[id - 1];
        }
      }
    {
      // boxes with a face toward another GPU (halo overlap in smooth_boxes)
      std::vector<int> bnd, in;
      for (int b = 0; b < L.n; b++) {
        bool r = false;
        for (int nb = 0; nb < 6; nb++) r |= L.h_nbk[(size_t)b * 6 + nb] == NB_REMOTE;
        (r ? bnd : in).push_back(b);
      }
      if (!bnd.empty()) {
        L.n_bnd = (int)bnd.size();
        L.n_int = (int)in.size();
        L.d_bnd = to_device(bnd);
        L.d_int = to_device(in);
        std::vector<uint8_t> isb(L.n, 0), push0(L.n, 0);
        for (int b : bnd) isb[b] = 1;
        for (int b : in)
          for (int nb = 0; nb < 6; nb++)
            if (L.h_nbk[(size_t)b * 6 + nb] == NB_LOCAL && isb[L.h_nba[(size_t)b * 6 + nb]]) push0[b] |= 1u << nb;
        L.d_push0 = to_device(push0);
        std::vector<int> bf;
        for (int b : bnd)
          for (int nb = 0; nb < 6; nb++)
            if (L.h_nbk[(size_t)b * 6 + nb] == NB_PHYS || L.h_nbk[(size_t)b * 6 + nb] == NB_RB) {
              bf.push_back(b);
              break;
            }
        L.n_bndface = (int)bf.size();
        L.d_bndface = to_device(bf);
      }
    }
    L.d_phi = L.d_data;
    build_block3(c, L);
    L.d_sendpos = to_device(sendpos);
    L.d_nbk = to_device(L.h_nbk);
    L.d_nba = to_device(L.h_nba);
    L.d_rb = to_device(L.h_rb);
    L.h_sendpos = sendpos;
    pack_topo(L);
    // parents / leaves (my_parents, my_leaves) as local indices
    for (int id : c->parents[l])
      if (owns(id)) L.parents.push_back(c->local_index[id]);
    for (int id : c->leaves[l])
      if (owns(id)) L.leaves.push_back(c->local_index[id]);
    L.d_parents = to_device(L.parents);
    L.d_leaves = to_device(L.leaves);
    {
      std::vector<uint8_t> pm(L.n, 0);
      for (int b : L.parents) pm[b] = 1;
      L.d_parmask = to_device(pm);
    }
    dmalloc(&L.d_scratch, sizeof(double) * L.leaves.size());
    dmalloc(&L.d_scratch_rhs, sizeof(double) * L.leaves.size());
    L.all_parents = L.n > 0 && (int)L.parents.size() == L.n;
  }
  // grid transfers between lvl-1 (coarse) and lvl (fine)
  for (int l = c->lowest + 1; l <= c->highest; l++) {
    Level& F = c->levels[l];
    Level& C = c->levels[l - 1];
    const int nc = F.nc, hnc = nc / 2;
    F.parent_local.assign(F.n, -1);
    F.dix_packed.assign(F.n, 0);
    std::vector<int> pairs;
    std::vector<Rec> rsend, rrecv, psend, precv;
    for (int b = 0; b < F.n; b++) {
      const int id = F.ids[b], p = T.parent(id);
      int d[3];
      T.child_offset(id, d);
      F.dix_packed[b] = pack_dix(d);
      int slot = 0;
      for (int s = 1; s <= 8; s++)
        if (T.child(p, s) == id) slot = s;
      if (owns(p)) {
        F.parent_local[b] = c->local_index[p];
        pairs.push_back(b);
        // a replicated parent of a distributed child: every peer restricts
        // into its own copy of the parent
        if (C.replicated && !F.replicated)
          for (int r = 0; r < c->n_ranks; r++)
            if (r != me) rsend.push_back({r, (long long)p * 8 + slot, b, 0});
      } else {
        rsend.push_back({T.rank(p), (long long)p * 8 + slot, b, 0});   // restrict_set_buffer
        precv.push_back({T.rank(p), (long long)id, b, 0});             // prolong_onto remote
      }
    }
    for (int pb = 0; pb < C.n; pb++) {
      const int p = C.ids[pb];
      for (int s = 1; s <= 8; s++) {
        const int ch = T.child(p, s);
        if (ch <= 0 || owns(ch)) continue;
        int d[3];
        T.child_offset(ch, d);
        rrecv.push_back({T.rank(ch), (long long)p * 8 + s, pb, pack_dix(d)});   // restrict_onto
        // (the child's owner holds a replicated parent itself)
        if (!C.replicated) psend.push_back({T.rank(ch), (long long)ch, pb, pack_dix(d)});   // prolong_set_buffer
      }
    }
    F.restr.send = group(rsend, 1);
    F.restr.recv = group(rrecv, 2);
    F.restr.send_ints = 1;
    F.restr.recv_ints = 2;
    F.restr.item_doubles = hnc * hnc * hnc;
    finalize_transfer(F.restr);
    F.prol.send = group(psend, 2);
    F.prol.recv = group(precv, 1);
    F.prol.send_ints = 2;
    F.prol.recv_ints = 1;
    F.prol.item_doubles = nc * nc * nc;
    finalize_transfer(F.prol);
    F.n_pairs = (int)pairs.size();
    F.d_pairs = to_device(pairs);
    F.d_parent_local = to_device(F.parent_local);
    F.d_dix = to_device(F.dix_packed);
    // k_prolong_smooth needs, for every same-GPU fine face whose neighbour has
    // another parent, that parent on this GPU as the coarse neighbour (boxes
    // with a face on another GPU are not fused)
    F.prolong_smooth_ok = F.n > 0 && F.n_pairs == F.n;
    const bool one_child = C.nc * 2 == F.nc;
    for (int b = 0; b < F.n && F.prolong_smooth_ok; b++) {
      bool remote = false;
      for (int nb = 0; nb < 6; nb++) remote |= F.h_nbk[(size_t)b * 6 + nb] == NB_REMOTE;
      if (remote) continue;   // takes correct + fill + the substep (prolong_smooth())
      int d[3];
      T.child_offset(F.ids[b], d);
      for (int nb = 1; nb <= 6; nb++) {
        const int kind = F.h_nbk[(size_t)b * 6 + nb - 1];
        if (kind == NB_PHYS || kind == NB_RB) continue;   // (formed from the box's own cells)
        if (kind != NB_LOCAL) { F.prolong_smooth_ok = false; break; }
        const bool low = nb & 1;
        const bool sib = !one_child && (low ? d[(nb - 1) >> 1] == F.nc / 2 : d[(nb - 1) >> 1] == 0);
        if (!sib && C.h_nbk[(size_t)F.parent_local[b] * 6 + nb - 1] != NB_LOCAL) {
          F.prolong_smooth_ok = false;
          break;
        }
      }
    }
    build_block3c(c, F, C);
  }
  // communication buffers, sized for the largest transfer touching each level
  if (c->n_ranks > 1) {
    std::map<int, size_t> sendn, recvn;
    for (int l = c->lowest; l <= c->highest; l++) {
      Level& L = c->levels[l];
      auto upd = [](std::map<int, size_t>& m, int k, size_t v) { m[k] = std::max(m[k], v); };
      upd(sendn, l, (size_t)L.halo.n_send * L.halo.item_doubles);
      upd(recvn, l, (size_t)L.halo.n_recv * L.halo.item_doubles);
      upd(sendn, l, (size_t)L.repl.n_send * L.repl.item_doubles);
      upd(recvn, l, (size_t)L.repl.n_recv * L.repl.item_doubles);
      upd(sendn, l, (size_t)L.deep_rhs.n_send * L.deep_rhs.item_doubles);
      upd(recvn, l, (size_t)L.deep_rhs.n_recv * L.deep_rhs.item_doubles);
      if (l > c->lowest) {
        upd(sendn, l, (size_t)L.restr.n_send * L.restr.item_doubles);      // fine side packs
        upd(recvn, l - 1, (size_t)L.restr.n_recv * L.restr.item_doubles);  // coarse side receives
        upd(sendn, l - 1, (size_t)L.prol.n_send * L.prol.item_doubles);    // coarse side packs
        upd(recvn, l, (size_t)L.prol.n_recv * L.prol.item_doubles);        // fine side receives
      }
    }
    for (int l = c->lowest; l <= c->highest; l++) {
      Level& L = c->levels[l];
      L.sendbuf_doubles = sendn[l];
      L.recvbuf_doubles = recvn[l];
      dmalloc(&L.d_sendbuf, sizeof(double) * sendn[l]);
      dmalloc(&L.d_recvbuf, sizeof(double) * recvn[l]);
      dmalloc(&L.d_rbsend, sizeof(double) * (size_t)L.rbx.n_send * L.rbx.item_doubles);
      dmalloc(&L.d_rbrecv, sizeof(double) * (size_t)L.rbx.n_recv * L.rbx.item_doubles);
    }
  }
  // k_gsrb3 / k_gsrb4's correction form on split levels: which path the
  // up-smoothing takes decides collective rounds (the deep halo of both
  // levels, deep_res), and whether the coarse records could be built depends
  // on each rank's boxes, so the ranks agree: every rank holding boxes of the
  // level must have them, else none uses them
  if (c->n_ranks > 1 && !c->host_only)
    for (int l = c->lowest + 1; l <= c->highest; l++) {
      Level& F = c->levels[l];
      if (!F.deep) continue;
      const bool fail = F.n > 0 && !F.d_b3c;
      if (allreduce(c, fail ? 1.0 : 0.0, true) > 0.5) dfree(F.d_b3c);
    }
  ensure_rhs_lex(c);
  rbh_build(c);
}

}  // namespace

// ===========================================================================
// C-ABI
extern "C" {

const char* omg_last_error(void) { return g_last_error.c_str(); }

int omg_get_unique_id(void* out) {
  return guarded([&] {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
  });
}

int omg_loopback_unique_id(long long tag, void* out) {
  return guarded([&] {
    std::memset(out, 0, OMG_UNIQUE_ID_BYTES);
    std::memcpy(out, kLoopMagic, sizeof(kLoopMagic));
    std::memcpy((char*)out + sizeof(kLoopMagic), &tag, sizeof(tag));
  });
}

int omg_host_unique_id(void* out) {
  return guarded([&] {
    std::memset(out, 0, OMG_UNIQUE_ID_BYTES);
    std::memcpy(out, kHostMagic, sizeof(kHostMagic));
  });
}

int omg_set_host_transport(omg_ctx* c, omg_host_exchange_fn exchange, omg_host_allgather_fn allgather, void* user) {
  return guarded([&] {
    if (!c->host_xport) throw OmgError("omg_set_host_transport: the context was not created with omg_host_unique_id");
    c->hx_exchange = exchange;
    c->hx_allgather = allgather;
    c->hx_user = user;
  });
}

int omg_device_count(int* n) {
  return guarded([&] { HIPCHK(hipGetDeviceCount(n)); });
}

int omg_ctx_create(omg_ctx** out, int device, int rank, int n_ranks, const void* unique_id) {
  return guarded([&] {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) throw OmgError("bad rank / n_ranks");
    if (n_ranks > 1 && !unique_id && device != OMG_DEVICE_NONE)
      throw OmgError("unique_id required for n_ranks > 1");
    // the switches the communication plan depends on (read by plan-only
    // contexts too, whose plans the CPU tests pair up)
    auto plan_switches = [](omg_ctx* c) {
      c->no_block3 = env_flag("OMG_NO_BLOCK3");
      c->no_block3_phys = env_flag("OMG_NO_BLOCK3_PHYS");
      c->no_deep = env_flag("OMG_NO_DEEP");
      // (tests: the smallest level k_gsrb3 serves; OMG_BLOCK3_MIN_BOXES)
      if (const char* v = getenv("OMG_BLOCK3_MIN_BOXES")) c->b3_min_boxes = std::max(1, atoi(v));
      // (tests: the column length, 2 .. 16 boxes, even; OMG_BLOCK3_COLUMN)
      if (const char* v = getenv("OMG_BLOCK3_COLUMN")) c->b3_col = std::min(std::max(2, atoi(v) & ~1), kB3MaxZ);
      if (const char* v = getenv("OMG_BLOCK3_SMALL_COL")) c->b3_col_small = std::min(std::max(2, atoi(v) & ~1), kB3MaxZ);
    };
    if (device == OMG_DEVICE_NONE) {   // plan-only context: no HIP, no RCCL
      omg_ctx* c = new omg_ctx();
      c->device = device;
      c->rank = rank;
      c->n_ranks = n_ranks;
      c->host_only = true;
      plan_switches(c);
      *out = c;
      return;
    }
    if (device < 0) {   // one rank per GPU: rank modulo the visible devices
      int n_dev = 0;
      HIPCHK(hipGetDeviceCount(&n_dev));
      if (n_dev < 1) throw OmgError("no HIP device visible");
      device = rank % n_dev;
    }
    omg_ctx* c = new omg_ctx();
    c->device = device;
    c->rank = rank;
    c->n_ranks = n_ranks;
    c->no_tail = env_flag("OMG_NO_TAIL");
    c->no_fuse_up = env_flag("OMG_NO_FUSE_UP");
    c->no_skip1 = env_flag("OMG_NO_SKIP1");
    c->tail_timing = env_flag("OMG_TAIL_TIMING");
    c->no_fill_tile = env_flag("OMG_NO_FILL_TILE");
    c->no_fill_crhs = env_flag("OMG_NO_FILL_CRHS");
    c->no_tail_crhs = env_flag("OMG_NO_TAIL_CRHS");
    c->no_rbgv = env_flag("OMG_NO_RBGV");
    c->no_graph = !env_flag("OMG_GRAPH");
    c->no_fuse_down = env_flag("OMG_NO_FUSE_DOWN");
    c->no_rb_fill_fuse = env_flag("OMG_NO_RB_FUSE");
    c->no_gs_plane = env_flag("OMG_NO_GS_PLANE");
    c->no_fill_xl = env_flag("OMG_NO_FILL_XL");
    c->no_gs_dbl = env_flag("OMG_NO_GS_DBL");
    plan_switches(c);
    c->no_block3p = env_flag("OMG_NO_BLOCK3P");
    c->no_block3r = env_flag("OMG_NO_BLOCK3R");
    c->block4 = !env_flag("OMG_NO_BLOCK4");
    c->no_block4p = env_flag("OMG_NO_BLOCK4P");
    c->block4_phys = env_flag("OMG_BLOCK4_PHYS");
    c->no_defer_gc = env_flag("OMG_NO_DEFER_GC");
    c->no_fuse_down_bc = env_flag("OMG_NO_FUSE_DOWN_BC");
    c->roctx = env_flag("OMG_ROCTX");
    c->debug = env_flag("OMG_DEBUG");
    // (on under OMG_DEBUG too: a rank that uploads phi alone would otherwise
    // make halo exchanges the others skip, a hang or mispaired messages)
    c->check_collective = env_flag("OMG_CHECK_COLLECTIVE") || c->debug;
    if (const char* v = getenv("OMG_GRAPH_FAIL")) c->graph_fail_at = std::atoi(v);   // tests only
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&c->d_scalar, sizeof(double) * (64 + 2 * (size_t)n_ranks)));
    HIPCHK(hipMalloc(&c->d_red, sizeof(double) * (8 + 2 * (size_t)n_ranks)));
    HIPCHK(hipMemset(c->d_red, 0, sizeof(double) * (8 + 2 * (size_t)n_ranks)));
    HIPCHK(hipMalloc(&c->d_maxslots, sizeof(unsigned long long) * omg::kMaxSlots * omg::kMaxSlotStride));
    // (allocated here: no allocation may happen while a cycle is captured)
    HIPCHK(hipMalloc(&c->d_tail, sizeof(TailArgs)));
    c->h_tail = new TailArgs;
    std::memset(c->h_tail, 0xff, sizeof(TailArgs));
    HIPCHK(hipMemset(c->d_maxslots, 0, sizeof(unsigned long long) * omg::kMaxSlots * omg::kMaxSlotStride));
    HIPCHK(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    {
      // the halo stream at the highest priority: its RCCL kernels are queued
      // behind the boundary boxes while an interior substep of thousands of
      // workgroups fills every CU; priority lets the dispatcher place them first
      int least = 0, greatest = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIPCHK(hipStreamCreateWithPriority(&c->stream_comm, hipStreamNonBlocking, greatest));
      c->comm_priority = greatest;
    }
    HIPCHK(hipEventCreateWithFlags(&c->ev_bnd, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_comm, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_side, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_phi, hipEventDisableTiming));
    HIPCHK(hipHostMalloc(&c->h_scalar, sizeof(double) * (16 + (size_t)n_ranks)));
    for (int iv = 0; iv < kMaxVars; iv++)
      for (int nb = 0; nb < 6; nb++) {
        c->bc[iv].type[nb] = OMG_BC_DIRICHLET;
        c->bc[iv].value[nb] = 0.0;
      }
    if (n_ranks > 1 && std::memcmp(unique_id, kLoopMagic, sizeof(kLoopMagic)) == 0) {
      long long tag;
      std::memcpy(&tag, (const char*)unique_id + sizeof(kLoopMagic), sizeof(tag));
      std::lock_guard<std::mutex> lk(g_loop_mu);
      auto& g = g_loops[tag];
      if (!g) {
        g = std::make_shared<omg_loop>();
        g->n_ranks = n_ranks;
      }
      if (g->n_ranks != n_ranks) throw OmgError("loopback group: n_ranks mismatch");
      c->loop = g;
    } else if (n_ranks > 1 && std::memcmp(unique_id, kHostMagic, sizeof(kHostMagic)) == 0) {
      c->host_xport = true;   // the callbacks come with omg_set_host_transport
    } else if (n_ranks > 1) {
      ncclUniqueId id;
      std::memcpy(&id, unique_id, sizeof(id));
      ncclComm_t comm;
      NCCLCHK(ncclCommInitRank(&comm, n_ranks, id, rank));
      c->nccl = comm;
    }
    *out = c;
  });
}

int omg_ctx_destroy(omg_ctx* c) {
  return guarded([&] {
    if (!c) return;
    if (c->host_only) {
      g_host_only = true;
      free_levels(c);
      g_host_only = false;
      delete c;
      return;
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream2);
    (void)hipStreamSynchronize(c->stream_comm);
    free_levels(c);
    dfree(c->d_scalar);
    if (c->d_tail) (void)hipFree(c->d_tail);
    if (c->d_tail_stamps) (void)hipFree(c->d_tail_stamps);
    delete c->h_tail;
    dfree(c->d_red);
    dfree(c->d_maxslots);
    for (auto& kv : c->graphs)
      if (kv.second) (void)hipGraphExecDestroy(kv.second);
    c->graphs.clear();
    dfree(c->d_stage);
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    if (c->ev_side) (void)hipEventDestroy(c->ev_side);
    if (c->ev_phi) (void)hipEventDestroy(c->ev_phi);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->stream_comm) (void)hipStreamDestroy(c->stream_comm);
    if (c->ev_bnd) (void)hipEventDestroy(c->ev_bnd);
    if (c->ev_comm) (void)hipEventDestroy(c->ev_comm);
    if (c->h_scalar) (void)hipHostFree(c->h_scalar);
    if (c->h_xsend) (void)hipHostFree(c->h_xsend);
    if (c->h_xrecv) (void)hipHostFree(c->h_xrecv);
    if (c->nccl) (void)ncclCommDestroy((ncclComm_t)c->nccl);
    if (c->loop) {   // the last context of a loopback group removes it
      std::lock_guard<std::mutex> lk(g_loop_mu);
      for (auto it = g_loops.begin(); it != g_loops.end(); ++it)
        if (it->second == c->loop && it->second.use_count() == 2) {
          g_loops.erase(it);
          break;
        }
      c->loop.reset();
    }
    (void)hipStreamDestroy(c->stream);
    delete c;
  });
}

int omg_tree_setup(omg_ctx* c, int n_boxes, const int* lvl, const int* parent, const int* children,
                   const int* neighbors, const int* ix, const int* rank, int lowest_lvl,
                   int highest_lvl, int first_normal_lvl, int box_size, const int* box_size_lvl,
                   const double* dr, const int* list_off, const int* lists, int n_vars) {
  return guarded([&] {
    if (n_vars < 4 || n_vars > kMaxVars) throw OmgError("n_vars out of range");
    struct HostOnly {
      explicit HostOnly(bool on) { g_host_only = on; }
      ~HostOnly() { g_host_only = false; }
    } host_only_scope(c->host_only);
    if (!c->host_only) (void)hipSetDevice(c->device);
    free_levels(c);
    c->n_boxes = n_boxes;
    c->lvl.assign(lvl, lvl + n_boxes);
    c->parent.assign(parent, parent + n_boxes);
    c->children.assign(children, children + 8 * (size_t)n_boxes);
    c->neighbors.assign(neighbors, neighbors + 6 * (size_t)n_boxes);
    c->ix.assign(ix, ix + 3 * (size_t)n_boxes);
    c->rank_of.assign(rank, rank + n_boxes);
    c->lowest = lowest_lvl;
    c->highest = highest_lvl;
    c->first_normal = first_normal_lvl;
    c->box_size = box_size;
    c->n_vars = n_vars;
    c->bsl.clear();
    c->drl.clear();
    c->ids.clear(); c->leaves.clear(); c->parents.clear(); c->ref_bnds.clear();
    for (int l = lowest_lvl; l <= highest_lvl; l++) {
      const int li = l - lowest_lvl;
      c->bsl[l] = box_size_lvl[li];
      c->drl[l] = {dr[3 * li], dr[3 * li + 1], dr[3 * li + 2]};
      std::map<int, std::vector<int>>* dst[4] = {&c->ids, &c->leaves, &c->parents, &c->ref_bnds};
      for (int t = 0; t < 4; t++) {
        const int a = list_off[4 * li + t], b = list_off[4 * li + t + 1];
        (*dst[t])[l] = std::vector<int>(lists + a, lists + b);
      }
    }
    if (!c->host_only) {
      host_sync(c, c->stream);
      host_sync(c, c->stream2);
    }
    c->rhs_cache_valid = false;
    c->phi_shift_pending = false;
    c->phi_mean_on_side = false;
    build_plan(c);
    if (!c->host_only) HIPCHK(hipDeviceSynchronize());
  });
}

int omg_plan_transfer(omg_ctx* c, int lvl, int which, int dir, int cap, int* peers, long long* keys,
                      int* n_items, int* item_doubles) {
  return guarded([&] {
    Level* L = level_ptr(c, lvl);
    if (!L) throw OmgError("no such level");
    if (which < 0 || which > 5) throw OmgError("omg_plan_transfer: bad transfer");
    const Transfer* T[6] = {&L->halo, &L->restr, &L->prol, &L->rbx, &L->repl, &L->deep_phi};
    const auto& lists = dir ? T[which]->recv : T[which]->send;
    int n = 0;
    for (auto& p : lists)
      for (long long k : p.keys) {
        if (n < cap) {
          peers[n] = p.peer;
          keys[n] = k;
        }
        n++;
      }
    *n_items = n;
    *item_doubles = T[which]->item_doubles;
  });
}

int omg_set_operator(omg_ctx* c, int op, double lambda) {
  return guarded([&] { set_operator(c, op, lambda); });
}

int omg_set_smoother(omg_ctx* c, int smoother, int n_cycle_down, int n_cycle_up, int max_coarse_cycles,
                     double res_abs, double res_rel) {
  return guarded([&] {
    if (smoother != OMG_SMOOTHER_GS && smoother != OMG_SMOOTHER_GSRB)
      throw OmgError("unsupported smoother type");
    c->smoother = smoother;
    c->n_substeps = smoother == OMG_SMOOTHER_GSRB ? 2 : 1;
    ensure_rhs_lex(c);
    c->n_cycle_down = n_cycle_down;
    c->n_cycle_up = n_cycle_up;
    c->max_coarse_cycles = max_coarse_cycles;
    c->res_abs = res_abs;
    c->res_rel = res_rel;
  });
}

int omg_set_subtract_mean(omg_ctx* c, int on) {
  return guarded([&] { c->subtract_mean = on; });
}

int omg_set_bc(omg_ctx* c, int iv, int nb, int bc_type, double bc_value) {
  return guarded([&] {
    phi_dirty_all(c);
    if (iv < 1 || iv > kMaxVars || nb < 1 || nb > 6) throw OmgError("omg_set_bc: bad iv/nb");
    c->bc[iv - 1].type[nb - 1] = bc_type;
    c->bc[iv - 1].value[nb - 1] = bc_value;
  });
}

int omg_set_bc_faces(omg_ctx* c, int iv, const long long* face_off, const int* face_type,
                     const double* data, long long n_data) {
  return guarded([&] {
    if (iv < 1 || iv > kMaxVars) throw OmgError("omg_set_bc_faces: bad iv");
    phi_dirty_all(c);
    const int k = iv - 1;
    for (auto& kv : c->d_face_off_lvl[k]) dfree(kv.second);
    for (auto& kv : c->d_face_type_lvl[k]) dfree(kv.second);
    c->d_face_off_lvl[k].clear();
    c->d_face_type_lvl[k].clear();
    c->h_face_off_lvl[k].clear();
    c->h_face_type_lvl[k].clear();
    dfree(c->d_face_data[k]);
    if (!face_off) return;
    // only the faces of my boxes travel to the device, re-packed
    std::vector<double> packed;
    for (auto& kv : c->levels) {
      Level& L = kv.second;
      if (!L.n) continue;
      std::vector<long long> off(L.n * 6, -1);
      std::vector<int> typ(L.n * 6, 0);
      const long long n2 = (long long)L.nc * L.nc;
      if (L.replicated) {
        // every copy needs the table: a face tabulated for one box of the
        // level must be tabulated for every box with that physical face
        bool any[6] = {}, miss[6] = {};
        for (int b = 0; b < L.n; b++)
          for (int nb = 0; nb < 6; nb++) {
            if (L.h_nbk[(size_t)b * 6 + nb] != NB_PHYS) continue;
            (face_off[(size_t)(L.ids[b] - 1) * 6 + nb] >= 0 ? any : miss)[nb] = true;
          }
        for (int nb = 0; nb < 6; nb++)
          if (any[nb] && miss[nb])
            throw OmgError("omg_set_bc_faces: replicated level " + std::to_string(L.lvl) +
                           " needs the boundary table of every box (omg_replicated_level)");
      }
      for (int b = 0; b < L.n; b++)
        for (int nb = 0; nb < 6; nb++) {
          const long long o = face_off[(size_t)(L.ids[b] - 1) * 6 + nb];
          if (o < 0) continue;
          if (o + n2 > n_data) throw OmgError("omg_set_bc_faces: offset out of range");
          off[b * 6 + nb] = (long long)packed.size();
          typ[b * 6 + nb] = face_type[(size_t)(L.ids[b] - 1) * 6 + nb];
          packed.insert(packed.end(), data + o, data + o + n2);
        }
      c->d_face_off_lvl[k][kv.first] = to_device(off);
      c->d_face_type_lvl[k][kv.first] = to_device(typ);
      c->h_face_off_lvl[k][kv.first] = off;
      c->h_face_type_lvl[k][kv.first] = typ;
    }
    c->d_face_data[k] = to_device(packed);
  });
}

int omg_level_size(omg_ctx* c, int lvl, int* n_boxes, int* nc) {
  return guarded([&] {
    Level* L = level_ptr(c, lvl);
    if (!L) throw OmgError("no such level");
    *n_boxes = (int)L->host_local.size();
    *nc = L->nc;
  });
}

int omg_set_coarse_replication(omg_ctx* c, long long max_cells) {
  return guarded([&] {
    if (!c->levels.empty()) throw OmgError("omg_set_coarse_replication: call before omg_tree_setup");
    if (max_cells < 0) throw OmgError("omg_set_coarse_replication: max_cells < 0");
    c->rep_cells = max_cells;
  });
}

int omg_replicated_level(omg_ctx* c, int* lvl) {
  return guarded([&] { *lvl = c->rep_lvl == INT_MIN ? c->lowest - 1 : c->rep_lvl; });
}

// staging buffer in the reference's box layout
double* stage(omg_ctx* c, size_t n) {
  if (n > c->stage_n) {
    dfree(c->d_stage);
    HIPCHK(hipMalloc(&c->d_stage, sizeof(double) * n));
    c->stage_n = n;
  }
  return c->d_stage;
}

int omg_upload_level(omg_ctx* c, int lvl, int iv, const double* host) {
  return guarded([&] {
    enter(c);
    Level* L = level_ptr(c, lvl);
    if (!L) throw OmgError("no such level");
    if (iv < 1 || iv > c->n_vars) throw OmgError("bad variable index");
    // (before the early return: a rank without boxes here still drops the
    // flag, which the multi-rank stand-alone fill decision relies on)
    if (iv == 1) phi_dirty(c, lvl);
    if (!L->n) return;
    const size_t s = L->nc + 2, box = s * s * s, n = box * L->n;
    double* st = stage(c, n);
    if (L->replicated) {
      // the host's boxes into their slots, then to every peer (collective)
      std::vector<double> full(n, 0.0);
      for (size_t q = 0; q < L->host_local.size(); q++)
        std::memcpy(full.data() + box * L->host_local[q], host + box * q, sizeof(double) * box);
      HIPCHK(hipMemcpyAsync(st, full.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
      launch_from_ref(L->view(), iv, st, c->stream);
      if (L->repl.n_send || L->repl.n_recv) {
        launch_box_pack(L->view(), iv, L->repl.d_send_items, L->repl.n_send, L->d_sendbuf, c->stream);
        exchange(c, L->repl, L->d_sendbuf, L->d_recvbuf, nullptr, lvl);
        launch_box_unpack(L->view(), iv, L->repl.d_recv_items, L->repl.n_recv, L->d_recvbuf, c->stream);
      }
      host_sync(c, c->stream);
      return;
    }
    HIPCHK(hipMemcpyAsync(st, host, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    launch_from_ref(L->view(), iv, st, c->stream);
    host_sync(c, c->stream);
  });
}

int omg_download_level(omg_ctx* c, int lvl, int iv, double* host) {
  return guarded([&] {
    enter(c, false);
    Level* L = level_ptr(c, lvl);
    if (!L) throw OmgError("no such level");
    if (iv < 1 || iv > c->n_vars) throw OmgError("bad variable index");
    if (!L->n) return;
    const size_t s = L->nc + 2, box = s * s * s, n = box * L->n;
    double* st = stage(c, n);
    launch_to_ref(L->view(), iv, st, c->debug ? snan_value() : 0.0, c->stream);
    if (L->replicated) {   // the host's boxes only
      std::vector<double> full(n);
      HIPCHK(hipMemcpyAsync(full.data(), st, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
      host_sync(c, c->stream);
      for (size_t q = 0; q < L->host_local.size(); q++)
        std::memcpy(host + box * q, full.data() + box * L->host_local[q], sizeof(double) * box);
      return;
    }
    HIPCHK(hipMemcpyAsync(host, st, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    host_sync(c, c->stream);
  });
}

int omg_fas_vcycle(omg_ctx* c, int highest_lvl, int want_max_res, double* max_res, int standalone) {
  return guarded([&] {
    const double r = run_cycle(c, 1 + (want_max_res ? 2 : 0) + 4 * (standalone != 0) + 8 * (highest_lvl + 64),
                               [&] { return fas_vcycle(c, highest_lvl, want_max_res != 0, standalone != 0); });
    if (want_max_res && max_res) *max_res = r;
    if (want_max_res) check_finite_res(r, "mg_fas_vcycle");
  });
}

int omg_fas_fmg(omg_ctx* c, int have_guess, int want_max_res, double* max_res) {
  return guarded([&] {
    const double r = run_cycle(c, 2 + (want_max_res ? 2 : 0) + 4 * (have_guess != 0),
                               [&] { return fas_fmg(c, have_guess != 0, want_max_res != 0); });
    if (want_max_res && max_res) *max_res = r;
    if (want_max_res) check_finite_res(r, "mg_fas_fmg");
  });
}

int omg_apply_op(omg_ctx* c, int i_out) {
  return guarded([&] { apply_op(c, i_out); });
}

int omg_set_rhs(omg_ctx* c, double f1, double f2) {
  return guarded([&] { set_rhs(c, f1, f2); });
}

int omg_diffusion_solve(omg_ctx* c, int op, double dt, double diffusion_coeff, int order, double max_res,
                        int* n_vcycles, double* res) {
  return guarded([&] { diffusion_solve(c, op, dt, diffusion_coeff, order, max_res, n_vcycles, res); });
}

int omg_restrict(omg_ctx* c, int iv) {
  return guarded([&] {
    enter(c);
    for (int l = c->highest; l >= c->lowest + 1; l--) restrict_lvl(c, iv, l);
  });
}
int omg_restrict_lvl(omg_ctx* c, int iv, int lvl) {
  return guarded([&] {
    enter(c);
    restrict_lvl(c, iv, lvl);
  });
}
int omg_fill_ghost_cells(omg_ctx* c, int iv) {
  return guarded([&] {
    enter(c);
    for (int l = c->lowest; l <= c->highest; l++) fill_gc_lvl(c, l, iv);
  });
}
int omg_fill_ghost_cells_lvl(omg_ctx* c, int lvl, int iv) {
  return guarded([&] {
    enter(c);
    fill_gc_lvl(c, lvl, iv);
  });
}
int omg_prolong(omg_ctx* c, int lvl, int iv, int iv_to, int add) {
  return guarded([&] {
    enter(c);
    prolong(c, lvl, iv, iv_to, add);
  });
}
int omg_smooth_boxes(omg_ctx* c, int lvl, int n_cycle) {
  return guarded([&] {
    enter(c);
    smooth_boxes(c, lvl, n_cycle);
  });
}
int omg_update_coarse(omg_ctx* c, int lvl) {
  return guarded([&] {
    enter(c);
    update_coarse(c, lvl);
  });
}
int omg_correct_children(omg_ctx* c, int lvl) {
  return guarded([&] {
    enter(c);
    correct_children(c, lvl);
  });
}
int omg_residual_lvl(omg_ctx* c, int lvl) {
  return guarded([&] {
    enter(c);
    residual_lvl(c, lvl, nullptr);
  });
}
int omg_max_residual_lvl(omg_ctx* c, int lvl, double* out) {
  return guarded([&] {
    enter(c);
    *out = max_residual_lvl(c, lvl);
    check_finite_res(*out, "max_residual_lvl");
  });
}
int omg_get_sum(omg_ctx* c, int iv, double* out) {
  return guarded([&] {
    enter(c, false);
    *out = get_sum(c, iv);
  });
}
int omg_subtract_mean(omg_ctx* c, int iv, int include_ghostcells) {
  return guarded([&] { subtract_mean(c, iv, include_ghostcells); });
}

// mg_phi_bc_store (m_ghost_cells.f90:66-117): the bc values of phi go into
// the rhs ghost cells and the bc type into the neighbour slot.
int omg_phi_bc_store(omg_ctx* c) {
  return guarded([&] {
    enter(c);
    phi_bc_store(c);
  });
}

int omg_poisson_free_3d(omg_ctx* c, int new_rhs, double max_fft_frac, int fmgcycle, int want_max_res,
                        double* max_res, const double* r_min, const double* box_r_min) {
  return guarded([&] {
    enter(c);
    const double r = poisson_free_3d(c, new_rhs != 0, max_fft_frac, fmgcycle != 0, want_max_res != 0, r_min,
                                     box_r_min);
    if (max_res && want_max_res) *max_res = r;
    if (want_max_res) check_finite_res(r, "mg_poisson_free_3d");
  });
}

int omg_free_planes(omg_ctx* c, int* fft_lvl, int* nx, double* planes, long long cap) {
  return guarded([&] {
    omg_free_state* S = c->free_state;
    if (!S || !S->initialized) throw OmgError("omg_free_planes: no free-space solve yet");
    *fft_lvl = S->fft_lvl;
    for (int d = 0; d < 3; d++) nx[d] = S->G.nx[d];
    const size_t n = 2 * ((size_t)nx[1] * nx[2] + (size_t)nx[0] * nx[2] + (size_t)nx[0] * nx[1]);
    if (planes && cap >= (long long)n) {
      HIPCHK(hipMemcpyAsync(planes, S->d_planes, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
      host_sync(c, c->stream);
    }
  });
}

int omg_comm_info(omg_ctx* c, int* n_ranks, int* transport) {
  return guarded([&] {
    if (c->nccl) {
      NCCLCHK(ncclCommCount((ncclComm_t)c->nccl, n_ranks));
      *transport = OMG_TRANSPORT_RCCL;
    } else if (c->loop) {
      *n_ranks = c->loop->n_ranks;
      *transport = OMG_TRANSPORT_LOOPBACK;
    } else if (c->host_xport) {
      *n_ranks = c->n_ranks;
      *transport = OMG_TRANSPORT_HOST;
    } else {
      *n_ranks = c->n_ranks;
      *transport = OMG_TRANSPORT_NONE;
    }
  });
}

int omg_synchronize(omg_ctx* c) {
  return guarded([&] {
    host_sync(c, c->stream);
    host_sync(c, c->stream2);
  });
}

void* omg_stream(omg_ctx* c) { return (void*)c->stream; }

int omg_set_refinement_bnd(omg_ctx* c, int iv, int nb, omg_rb_fn fn, void* user) {
  return guarded([&] {
    if (iv < 1 || iv > kMaxVars || nb < 1 || nb > 6) throw OmgError("omg_set_refinement_bnd: bad iv/nb");
    if (c->rb_fn[iv - 1][nb - 1] == (void*)fn && c->rb_user[iv - 1][nb - 1] == user) return;
    if (!c->host_only) HIPCHK(hipStreamSynchronize(c->stream));   // (staging buffers in use)
    c->rb_fn[iv - 1][nb - 1] = (void*)fn;
    c->rb_user[iv - 1][nb - 1] = fn ? user : nullptr;
    rbh_build(c);
  });
}

int omg_host_sync_count(omg_ctx* c, long long* n) {
  return guarded([&] { *n = c->n_host_syncs; });
}

int omg_comm_stream_priority(omg_ctx* c, int* priority) {
  return guarded([&] { *priority = c->comm_priority; });
}

int omg_set_profiling(omg_ctx* c, int on) {
  return guarded([&] {
    resolve_stats(c);
    c->profiling = on != 0;
  });
}

int omg_kernel_stats(omg_ctx* c, const char* name, long long* launches, double* total_ms, double* cells) {
  return guarded([&] {
    resolve_stats(c);
    auto it = c->stats.find(name);
    if (it == c->stats.end()) {
      *launches = 0;
      *total_ms = 0;
      *cells = 0;
      return;
    }
    *launches = it->second.launches;
    *total_ms = it->second.ms;
    *cells = it->second.cells;
  });
}

int omg_reset_stats(omg_ctx* c) {
  return guarded([&] {
    resolve_stats(c);
    c->stats.clear();
  });
}

}  // extern "C"
