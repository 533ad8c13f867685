// fake_dev.cpp -- TEST INFRASTRUCTURE ONLY: a CPU "device" for slab_core.hpp,
// so that the multi-GPU slab job's round and exchange logic -- the very code
// csrc/slab.hip runs on the 8-GPU node -- runs under `pytest -m "not gpu"`.
//
//   memory     host allocations in the library's padded layout (the same
//              stencil_layout arithmetic as api.hip's stencil_layout_init)
//   streams    synchronous: every operation completes when it is issued, so
//              events are host timestamps and waits are no-ops; what is
//              checked is the data flow -- which planes each round sweeps,
//              sends, receives and restores -- not stream concurrency
//   sweeps     stencil_sweepk's contract (K fused sweeps of [begin, end), halo
//              planes advanced, ghost cells never written) computed with the
//              ORACLE (oracle/oracle.c): the planes [begin - K r, end + K r)
//              are cut out as a dense ghost-padded sub-grid and swept K times;
//              the cut ends stand still like ghost planes, which reaches K r
//              planes inward after K sweeps and so never [begin, end)
//   face-signalled launches: the sweep plus one add per face to the counters
//   communicator: a mailbox, one FIFO per (communicator id, sender,
//              receiver) -- sends are buffered copies, receives match in
//              posting order as NCCL's do, a group's receives complete at its
//              end (blocking, with a timeout instead of a hang).  In memory for
//              the ranks of one process (rank-mode jobs in threads join by
//              their id); with FAKE_SLAB_MAILBOX_DIR set, files in that
//              directory (one per message, written then renamed), so ranks in
//              separate processes -- bench.py's gloo-launched ranks in the CPU
//              tests -- exchange their halos too
//
// Exported with the fake_slab_ prefix and the stencil_slab_* signatures
// (tests/cpu_slab/binding.py maps them onto stencil_amd.engine.SlabJob).
// Never linked into the product: it links liboracle.so.
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <fstream>
#include <sstream>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "oracle.h"
#include "slab_core.hpp"

namespace stencil {

namespace {
thread_local int g_code = STENCIL_OK;
thread_local char g_msg[512] = "";
}  // namespace

int set_error(int code, const char* fmt, ...) {
    g_code = code;
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_msg, sizeof g_msg, fmt, ap);
    va_end(ap);
    return code;
}
void clear_error() {
    g_code = STENCIL_OK;
    g_msg[0] = '\0';
}

namespace fake {

int g_k = 0;                          // sweeps per round (0: the library's rule)
bool g_signal = true;                 // face-signalled rounds allowed
int64_t g_free = int64_t(1) << 40;    // "device" free bytes (rolling margin from memory)
std::mutex g_stat_mu;
int64_t g_sweeps = 0, g_signal_sweeps = 0, g_sends = 0, g_recvs = 0, g_peer_copies = 0;
int64_t g_gated = 0, g_gate_bad = 0, g_xdone = 0;  // gated launches, numbering violations, completion stores

struct Event {
    std::chrono::steady_clock::time_point t{};
};

struct Mailbox {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::tuple<std::string, int, int>, std::deque<std::vector<char>>> q;
    std::map<std::string, int> joined;  // rank-mode communicators per id
};
Mailbox& mailbox() {
    static Mailbox m;
    return m;
}

struct Comm {
    std::string id;
    int rank = 0, nranks = 1;
    int64_t timeout_ms = 20000;  // a receive waits this long (the job's timeout)
    int64_t sent = 0;            // sends posted (FAKE_SLAB_MUTE_*)
};

// Test hook: FAKE_SLAB_MUTE_RANK=r, FAKE_SLAB_MUTE_AFTER=n -- rank r stops
// posting its sends after its first n (a peer that stopped answering).
bool muted(Comm* c) {
    const char* r = std::getenv("FAKE_SLAB_MUTE_RANK");
    if (!r || !*r || std::atoi(r) != c->rank) return false;
    const char* n = std::getenv("FAKE_SLAB_MUTE_AFTER");
    return c->sent++ >= (n && *n ? std::atoll(n) : 0);
}

struct PendingRecv {
    void* p;
    size_t bytes;
    int peer;
    Comm* c;
};
thread_local int t_group = 0;
thread_local std::vector<PendingRecv> t_pending;

// ---- the cross-process form: FAKE_SLAB_MAILBOX_DIR
const char* mail_dir() {
    const char* d = std::getenv("FAKE_SLAB_MAILBOX_DIR");
    return d && *d ? d : nullptr;
}
std::string hex_of(const std::string& id) {
    static const char* k = "0123456789abcdef";
    std::string h;
    for (unsigned char ch : id) {
        if (!ch) break;
        h += k[ch >> 4];
        h += k[ch & 15];
    }
    return h.substr(0, 48);
}
// per (id, from, to) message counters of THIS process (sends / receives)
std::mutex g_seq_mu;
std::map<std::tuple<std::string, int, int>, int64_t> g_sent, g_taken;
std::string mail_path(const std::string& id, int from, int to, int64_t seq) {
    std::ostringstream o;
    o << mail_dir() << "/m_" << hex_of(id) << "_" << from << "_" << to << "_" << seq;
    return o.str();
}
int file_send(const void* p, size_t bytes, int from, int to, const std::string& id) {
    int64_t seq;
    {
        std::lock_guard<std::mutex> lk(g_seq_mu);
        seq = g_sent[std::make_tuple(id, from, to)]++;
    }
    const std::string path = mail_path(id, from, to, seq), tmp = path + ".tmp";
    {
        std::ofstream f(tmp, std::ios::binary);
        f.write(static_cast<const char*>(p), std::streamsize(bytes));
        if (!f) return set_error(STENCIL_EHIP, "fake send: cannot write %s", tmp.c_str());
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) return set_error(STENCIL_EHIP, "fake send: rename failed");
    return STENCIL_OK;
}
int file_take(void* p, size_t bytes, int from, int to, const std::string& id, int64_t timeout_ms) {
    int64_t seq;
    {
        std::lock_guard<std::mutex> lk(g_seq_mu);
        seq = g_taken[std::make_tuple(id, from, to)]++;
    }
    const std::string path = mail_path(id, from, to, seq);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    while (access(path.c_str(), F_OK) != 0) {
        if (std::chrono::steady_clock::now() > deadline)
            return set_error(STENCIL_ETIMEOUT, "fake recv: rank %d waited %lld ms for rank %d", to,
                             (long long)timeout_ms, from);
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (size_t(f.tellg()) != bytes) return set_error(STENCIL_EHIP, "fake recv: %zu bytes posted, message differs", bytes);
    f.seekg(0);
    f.read(static_cast<char*>(p), std::streamsize(bytes));
    f.close();
    std::remove(path.c_str());
    return STENCIL_OK;
}

int take(void* p, size_t bytes, int peer, Comm* c) {
    if (mail_dir()) return file_take(p, bytes, peer, c->rank, c->id, c->timeout_ms);
    Mailbox& m = mailbox();
    std::unique_lock<std::mutex> lk(m.mu);
    const auto key = std::make_tuple(c->id, peer, c->rank);
    if (!m.cv.wait_for(lk, std::chrono::milliseconds(c->timeout_ms), [&] { return !m.q[key].empty(); }))
        return set_error(STENCIL_ETIMEOUT, "fake recv: rank %d waited %lld ms for rank %d", c->rank,
                         (long long)c->timeout_ms, peer);
    std::vector<char> msg = std::move(m.q[key].front());
    m.q[key].pop_front();
    if (msg.size() != bytes)
        return set_error(STENCIL_EHIP, "fake recv: %zu bytes posted, %zu sent", bytes, msg.size());
    std::memcpy(p, msg.data(), bytes);
    return STENCIL_OK;
}

}  // namespace fake

// a fake stream: synchronous, it only remembers its CU budget (the
// exchange's CU budget tuning: FAKE_SLAB_WIRE_MS below)
struct FStream {
    int cus = 0;
};

struct FakeDev {
    using Stream = FStream*;
    using Event = fake::Event*;
    using Comm = fake::Comm*;

    static int set_device(int) { return STENCIL_OK; }
    // api.hip's stencil_layout_init arithmetic (the rows padded so interior
    // x = 0 sits on a 128-B boundary)
    static int layout_init(const stencil_problem* p, stencil_layout* out) {
        if (!p || p->dims != 3 || p->radius < 1 || p->nx < 0 || p->ny < 0 || p->nz < 0 ||
            (p->halo > 0 && p->halo < p->radius))
            return set_error(STENCIL_EINVAL, "fake layout: bad problem");
        const int64_t r = p->radius, es = p->dtype == STENCIL_F32 ? 4 : 8;
        const int64_t align = 128 / es;
        const int64_t origin_x = (r + align - 1) / align * align;
        stencil_layout l{};
        l.prob = *p;
        l.row = (origin_x + p->nx + r + align - 1) / align * align;
        {  // api.hip's pitch rule (pitch_pad_bytes)
            const int64_t pitch = l.row * es, r = pitch % 32768;
            if (pitch >= 32768 - 512)
                l.row += (pitch >= 32768 && r <= 256 ? 384 - r : r >= 32768 - 512 ? 128 : 0) / es;
        }
        l.rows = p->ny + 2 * r;
        l.plane = l.row * l.rows;
        l.zghost = std::max<int64_t>(r, p->halo);
        l.planes = p->nz + 2 * l.zghost;
        l.origin = l.zghost * l.plane + r * l.row + origin_x;
        l.elems = l.plane * l.planes;
        l.bytes = l.elems * es;
        *out = l;
        return STENCIL_OK;
    }
    // iterate_tk_steps / iterate_box_steps of api.hip, unless a test sets K
    static int fuse_depth(const stencil_problem& p) {
        if (fake::g_k > 0) return fake::g_k;
        if (p.shape == STENCIL_BOX) return p.nx * p.ny >= int64_t(384) * 384 ? 4 : 3;
        return p.dtype == STENCIL_F32 && p.nx * p.ny >= (int64_t(1) << 20) ? 5 : 4;
    }
    static bool signal_enabled() { return fake::g_signal; }
    // the fake has no CUs: FAKE_SLAB_CONFINE=1 treats every slab as a grid of
    // several rounds of workgroups (staged rounds, unless STENCIL_SLAB_STAGED=0)
    static bool confine_exchange(const stencil_layout&, int) {
        const char* v = std::getenv("FAKE_SLAB_CONFINE");
        return v && std::atoi(v) != 0;
    }
    // the placement search's allocation and choice logic (timings are the
    // host's): STENCIL_SLAB_PLACEMENTS as the product reads it (default 1),
    // or FAKE_SLAB_PLACE=n
    static int placement_trials() {
        const char* v = std::getenv("FAKE_SLAB_PLACE");
        if (!v || !*v) v = std::getenv("STENCIL_SLAB_PLACEMENTS");
        return v && std::atoi(v) > 1 ? std::atoi(v) : 1;
    }
    static bool placement_verbose() { return false; }
    static bool staged_rounds() {
        const char* v = std::getenv("STENCIL_SLAB_STAGED");
        return !(v && *v && std::atoi(v) == 0);
    }
    // FAKE_SLAB_WIRE_MS=t: every exchange first sleeps t / cus ms on an
    // exchange stream confined to `cus` CUs per XCD (t * cus with
    // FAKE_SLAB_WIRE_INVERT=1): the tuning rounds then see the alternative
    // budget faster (or slower) and keep it (or not)
    static int wire_delay(Stream s, size_t) {
        const char* v = std::getenv("FAKE_SLAB_WIRE_MS");
        if (!v || std::atof(v) <= 0) return STENCIL_OK;
        const int c = std::max(1, s ? s->cus : 1);
        const char* inv = std::getenv("FAKE_SLAB_WIRE_INVERT");
        const double ms = (inv && std::atoi(inv)) ? std::atof(v) * c : std::atof(v) / c;
        std::this_thread::sleep_for(std::chrono::microseconds(int64_t(ms * 1000)));
        return STENCIL_OK;
    }
    static int xcu() { return 1; }
    static int xcu_alt() {
        const char* v = std::getenv("STENCIL_SLAB_XCU_ALT");
        return v && *v ? std::max(0, std::atoi(v)) : 4;
    }
    static int free_bytes(int64_t* out) {
        *out = fake::g_free;
        return STENCIL_OK;
    }
    static int alloc(int64_t bytes, void** p) {
        *p = std::calloc(size_t(bytes), 1);
        return *p ? STENCIL_OK : set_error(STENCIL_ENOMEM, "fake alloc of %lld bytes", (long long)bytes);
    }
    static void free(void* p) { std::free(p); }
    static int alloc_counters(uint32_t** c) {
        *c = static_cast<uint32_t*>(std::calloc(4, sizeof(uint32_t)));
        return *c ? STENCIL_OK : set_error(STENCIL_ENOMEM, "fake counters");
    }
    static void free_counters(uint32_t* c) { std::free(c); }
    static int alloc_flag(uint32_t** f) {
        *f = static_cast<uint32_t*>(std::calloc(1, sizeof(uint32_t)));
        return *f ? STENCIL_OK : set_error(STENCIL_ENOMEM, "fake flag");
    }
    static void free_flag(uint32_t* f) { std::free(f); }
    static int reset_counters(uint32_t* c, uint32_t* flag, uint64_t*) {
        if (c) std::memset(c, 0, 4 * sizeof(uint32_t));
        if (flag) *flag = 0;
        return STENCIL_OK;
    }
    static void release_waits(uint32_t* flag, uint64_t*) {
        if (flag) *flag = 1;
    }
    static int stream_create(Stream* s, int role, bool confine, int cus = -1) {
        *s = new FStream;
        (*s)->cus = confine && role == slab::STREAM_EXCHANGE ? (cus >= 0 ? cus : xcu()) : 0;
        return STENCIL_OK;
    }
    static void stream_destroy(Stream s) { delete s; }
    static int stream_sync(Stream) { return STENCIL_OK; }
    // synchronous streams: everything has completed when it was issued (a
    // receive that never arrives fails at issue, after the comm's timeout)
    static int sync_until(Stream, Comm, slab::Clock::time_point) { return STENCIL_OK; }
    static int event_sync_until(Event, Comm, slab::Clock::time_point) { return STENCIL_OK; }
    static int default_timeout_ms() {
        const char* v = std::getenv("STENCIL_SLAB_TIMEOUT_MS");
        return v && std::atoi(v) > 0 ? std::atoi(v) : 20000;
    }
    static int event_create(Event* e, bool) {
        *e = new fake::Event;
        return STENCIL_OK;
    }
    static void event_destroy(Event e) { delete e; }
    static int event_record(Event e, Stream) {
        e->t = std::chrono::steady_clock::now();
        return STENCIL_OK;
    }
    static int stream_wait(Stream, Event) { return STENCIL_OK; }
    static int debug_delay(Stream, int) { return STENCIL_OK; }  // copies are synchronous here
    static bool pull_wait_enabled() { return true; }
    static int debug_signal_skew() { return 0; }
    static int event_elapsed(float* ms, Event a, Event b) {
        *ms = std::chrono::duration<float, std::milli>(b->t - a->t).count();
        return STENCIL_OK;
    }

    // ---- the sweep: stencil_sweepk's contract through the oracle
    template <typename T>
    static int sweep_t(const stencil_layout* l, const T* src, T* dst, int64_t b, int64_t e, int k) {
        const stencil_problem& p = l->prob;
        const int64_t r = p.radius, zg = l->zghost, n = p.nz;
        const int64_t lo_bound = (p.flags & STENCIL_HALO_LO) ? -zg : -r;
        const int64_t hi_bound = (p.flags & STENCIL_HALO_HI) ? n + zg : n + r;
        const int64_t zlo = std::max(b - int64_t(k) * r, lo_bound), zhi = std::min(e + int64_t(k) * r, hi_bound);
        oracle_problem op{};
        op.dims = 3;
        op.dtype = p.dtype == STENCIL_F64 ? ORACLE_F64 : ORACLE_F32;
        op.shape = p.shape == STENCIL_BOX ? ORACLE_BOX : ORACLE_STAR;
        op.radius = int32_t(r);
        op.order = ORACLE_ORDER_NAIVE;
        op.nx = p.nx;
        op.ny = p.ny;
        op.nz = (zhi - zlo) - 2 * r;
        if (op.nz < e - b) return set_error(STENCIL_EINVAL, "fake sweep: range [%lld, %lld) beyond the readable planes",
                                           (long long)b, (long long)e);
        const int64_t sx = p.nx + 2 * r, sy = p.ny + 2 * r;
        std::vector<T> A(size_t(sx * sy * (zhi - zlo))), B;
        for (int64_t z = zlo; z < zhi; ++z)
            for (int64_t y = -r; y < p.ny + r; ++y)
                std::memcpy(&A[size_t(((z - zlo) * sy + (y + r)) * sx)], src + l->origin + z * l->plane + y * l->row - r,
                            size_t(sx) * sizeof(T));
        B = A;
        const int in_b = oracle_run(&op, uint32_t(k), A.data(), B.data(), 1);
        if (in_b < 0) return set_error(STENCIL_EINVAL, "fake sweep: oracle error %d", in_b);
        const std::vector<T>& R = in_b ? B : A;
        for (int64_t z = b; z < e; ++z)
            for (int64_t y = 0; y < p.ny; ++y)
                std::memcpy(dst + l->origin + z * l->plane + y * l->row, &R[size_t(((z - zlo) * sy + (y + r)) * sx + r)],
                            size_t(p.nx) * sizeof(T));
        return STENCIL_OK;
    }
    static int sweepk(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k, Stream) {
        if (b < 0 || e > l->prob.nz || b > e || k < 1) return set_error(STENCIL_EINVAL, "fake sweep: bad range");
        {
            std::lock_guard<std::mutex> lk(fake::g_stat_mu);
            ++fake::g_sweeps;
        }
        if (b == e) return STENCIL_OK;
        return l->prob.dtype == STENCIL_F64
                   ? sweep_t(l, static_cast<const double*>(src), static_cast<double*>(dst), b, e, k)
                   : sweep_t(l, static_cast<const float*>(src), static_cast<float*>(dst), b, e, k);
    }
    static bool rolling_overlap() {
        const char* v = std::getenv("STENCIL_SLAB_ROLLING_OVERLAP");
        return !(v && *v && std::atoi(v) == 0);
    }
    static bool serial_rounds() { return std::getenv("STENCIL_SLAB_SERIAL") && std::atoi(std::getenv("STENCIL_SLAB_SERIAL")); }
    static int face_signal_create(uint64_t** fs) {  // the fake waits synchronously: no signal word
        *fs = nullptr;
        return STENCIL_OK;
    }
    static void face_signal_destroy(uint64_t*) {}
    static int wait_face_signal(uint64_t*, uint64_t, Stream) { return STENCIL_OK; }
    static int sweepk_signal(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k,
                             uint32_t* counters, uint64_t*, int* nsig, Stream s) {
        if (int rc = sweepk(l, src, dst, b, e, k, s)) return rc;
        {
            std::lock_guard<std::mutex> lk(fake::g_stat_mu);
            ++fake::g_signal_sweeps;
        }
        counters[0] += 1;  // one add per face and launch (the faces are stored)
        counters[1] += 1;
        *nsig = 1;
        return STENCIL_OK;
    }
    // halo-gated launches (FAKE_SLAB_GATE=0: off): the fake's streams are
    // synchronous, so the exchange a gated launch waits for has completed
    // when the launch is issued -- unless the core's exchange numbering is
    // wrong, which counts as a violation (on a GPU: a launch that waits for
    // an exchange that never comes, or reads halos too early)
    static bool halo_gate(const stencil_layout&, int, bool) {
        const char* v = std::getenv("FAKE_SLAB_GATE");
        return !(v && *v && std::atoi(v) == 0);
    }
    static int sweepk_signal_gated(const stencil_layout* l, const void* src, void* dst, int64_t b, int64_t e, int k,
                                   uint32_t* counters, uint64_t* fsig, uint32_t need, uint32_t*, int* nsig, Stream s) {
        {
            std::lock_guard<std::mutex> lk(fake::g_stat_mu);
            ++fake::g_gated;
            if (int32_t(counters[3] - need) < 0 || counters[3] != need) ++fake::g_gate_bad;
        }
        return sweepk_signal(l, src, dst, b, e, k, counters, fsig, nsig, s);
    }
    static int exchange_done(uint32_t* counters, uint32_t value, Stream) {
        std::lock_guard<std::mutex> lk(fake::g_stat_mu);
        if (value != counters[3] + 1) ++fake::g_gate_bad;  // one completion per exchange, in order
        counters[3] = value;
        ++fake::g_xdone;
        return STENCIL_OK;
    }
    static int wait_counters(uint32_t* c, uint32_t* flag, uint32_t lo, uint32_t hi, Stream) {
        if (c[0] < lo || c[1] < hi) *flag = 1;  // synchronous: a count short now never arrives
        return STENCIL_OK;
    }
    static int read_timeout(uint32_t* flag, bool* timed_out) {
        *timed_out = *flag != 0;
        return STENCIL_OK;
    }
    static int copy_d2d(void* dst, const void* src, size_t bytes, Stream) {
        std::memmove(dst, src, bytes);
        return STENCIL_OK;
    }
    static int copy_peer(void* dst, int, const void* src, int, size_t bytes, Stream) {
        std::memmove(dst, src, bytes);
        std::lock_guard<std::mutex> lk(fake::g_stat_mu);
        ++fake::g_peer_copies;
        return STENCIL_OK;
    }
    // api.hip's fill_initial_kernel: padding 0, x-ghosts 1 at every y and z,
    // interior 0 or splitmix64(seed + linear index) (the oracle's u01)
    template <typename T>
    static void fill_t(const stencil_layout* l, T* g, int kind, uint64_t seed) {
        const stencil_problem& p = l->prob;
        const int64_t r = p.radius, ox = l->origin % l->row;
        for (int64_t pz = 0; pz < l->planes; ++pz)
            for (int64_t py = 0; py < l->rows; ++py)
                for (int64_t px = 0; px < l->row; ++px) {
                    const int64_t x = px - ox, y = py - r, z = pz - l->zghost;
                    T v = T(0);
                    if (x >= -r && x < p.nx + r) {
                        const bool xghost = x < 0 || x >= p.nx;
                        const bool interior = !xghost && y >= 0 && y < p.ny && z >= 0 && z < p.nz;
                        if (xghost) {
                            v = T(1);
                        } else if (interior && kind == STENCIL_INIT_RANDOM) {
                            uint64_t u = seed + uint64_t((z * p.ny + y) * p.nx + x);
                            u += 0x9e3779b97f4a7c15ULL;
                            u = (u ^ (u >> 30)) * 0xbf58476d1ce4e5b9ULL;
                            u = (u ^ (u >> 27)) * 0x94d049bb133111ebULL;
                            u ^= u >> 31;
                            v = sizeof(T) == 4 ? T(float(u >> 40) * 0x1.0p-24f) : T(double(u >> 11) * 0x1.0p-53);
                        }
                    }
                    g[(pz * l->rows + py) * l->row + px] = v;
                }
    }
    static int fill_initial(const stencil_layout* l, void* g, int kind, uint64_t seed, Stream) {
        if (l->prob.dtype == STENCIL_F64)
            fill_t(l, static_cast<double*>(g), kind, seed);
        else
            fill_t(l, static_cast<float*>(g), kind, seed);
        return STENCIL_OK;
    }
    // api.hip's copy_grid: host planes z = -r .. nz+r-1, x/y ghosts included
    static int copy_grid(const stencil_layout* l, void* g, const void* hs, void* hd, int64_t row, int64_t rows) {
        const stencil_problem& p = l->prob;
        const int64_t r = p.radius;
        const size_t es = p.dtype == STENCIL_F64 ? 8 : 4;
        const int64_t width = p.nx + 2 * r, height = p.ny + 2 * r;
        if (row < width || rows < height) return set_error(STENCIL_EINVAL, "host array too small");
        for (int64_t hz = 0; hz < p.nz + 2 * r; ++hz)
            for (int64_t y = 0; y < height; ++y) {
                char* d = static_cast<char*>(g) + size_t(l->origin + (hz - r) * l->plane + (y - r) * l->row - r) * es;
                const size_t h = size_t((hz * rows + y) * row) * es;
                if (hs)
                    std::memcpy(d, static_cast<const char*>(hs) + h, size_t(width) * es);
                else
                    std::memcpy(static_cast<char*>(hd) + h, d, size_t(width) * es);
            }
        return STENCIL_OK;
    }
    static int upload(const stencil_layout* l, void* g, const void* h, int64_t row, int64_t rows, Stream) {
        return copy_grid(l, g, h, nullptr, row, rows);
    }
    static int download(const stencil_layout* l, const void* g, void* h, int64_t row, int64_t rows, Stream) {
        return copy_grid(l, const_cast<void*>(g), nullptr, h, row, rows);
    }
    static int plane_sums(const stencil_layout* l, const void* g, double* out, Stream) {
        const stencil_problem& p = l->prob;
        for (int64_t z = 0; z < p.nz; ++z) {
            double acc = 0;
            for (int64_t y = 0; y < p.ny; ++y)
                for (int64_t x = 0; x < p.nx; ++x) {
                    const int64_t i = l->origin + z * l->plane + y * l->row + x;
                    acc += p.dtype == STENCIL_F64 ? static_cast<const double*>(g)[i]
                                                  : double(static_cast<const float*>(g)[i]);
                }
            out[z] = acc;
        }
        return STENCIL_OK;
    }

    // ---- the communicator
    static bool comm_available() { return true; }
    static int comm_init_all(Comm* comms, int n, const int*) {
        std::random_device rd;
        const std::string id = "all:" + std::to_string(rd()) + ":" + std::to_string(rd());
        for (int i = 0; i < n; ++i) comms[i] = new fake::Comm{id, i, n};
        return STENCIL_OK;
    }
    // as HipDev: a rank that never joins fails the collective with STENCIL_ETIMEOUT after timeout_ms
    static int comm_init_rank(Comm* comm, int nranks, const void* id, int rank, int64_t timeout_ms) {
        const std::string key(static_cast<const char*>(id), STENCIL_SLAB_ID_BYTES);
        if (fake::mail_dir()) {  // ranks in separate processes: a join file each, wait for all
            const std::string base = std::string(fake::mail_dir()) + "/join_" + fake::hex_of(key) + "_";
            std::ofstream(base + std::to_string(rank)) << rank;
            for (int r = 0; r < nranks; ++r)
                for (int it = 0; access((base + std::to_string(r)).c_str(), F_OK) != 0; ++it) {
                    if (it > timeout_ms)
                        return set_error(STENCIL_ETIMEOUT, "fake comm init: rank %d did not join within %lld ms", r,
                                         (long long)timeout_ms);
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                }
            *comm = new fake::Comm{key, rank, nranks};
            return STENCIL_OK;
        }
        fake::Mailbox& m = fake::mailbox();
        std::unique_lock<std::mutex> lk(m.mu);
        ++m.joined[key];
        m.cv.notify_all();
        // a collective, as ncclCommInitRank: every rank of the id must arrive
        if (!m.cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return m.joined[key] >= nranks; }))
            return set_error(STENCIL_ETIMEOUT, "fake comm init: %d of %d ranks joined within %lld ms", m.joined[key],
                             nranks, (long long)timeout_ms);
        *comm = new fake::Comm{key, rank, nranks};
        return STENCIL_OK;
    }
    static void comm_destroy(Comm c) { delete c; }
    static void comm_abort(Comm c) { delete c; }  // as ncclCommAbort: the comm is gone
    static void comm_set_timeout(Comm c, int64_t ms) { c->timeout_ms = ms; }
    static int group_start() {
        ++fake::t_group;
        return STENCIL_OK;
    }
    static int group_end() {
        if (fake::t_group <= 0) return set_error(STENCIL_EINVAL, "fake group_end without group_start");
        if (--fake::t_group > 0) return STENCIL_OK;
        std::vector<fake::PendingRecv> pend;
        pend.swap(fake::t_pending);
        for (const fake::PendingRecv& r : pend)
            if (int rc = fake::take(r.p, r.bytes, r.peer, r.c)) return rc;
        return STENCIL_OK;
    }
    static int send(const void* p, size_t bytes, int peer, Comm c, Stream) {
        if (peer < 0 || peer >= c->nranks) return set_error(STENCIL_EINVAL, "fake send to rank %d of %d", peer, c->nranks);
        if (fake::muted(c)) return STENCIL_OK;  // the test's silent peer
        if (fake::mail_dir()) {
            std::lock_guard<std::mutex> lk(fake::g_stat_mu);
            ++fake::g_sends;
            return fake::file_send(p, bytes, c->rank, peer, c->id);
        }
        fake::Mailbox& m = fake::mailbox();
        {
            std::lock_guard<std::mutex> lk(m.mu);
            m.q[std::make_tuple(c->id, c->rank, peer)].emplace_back(static_cast<const char*>(p),
                                                                    static_cast<const char*>(p) + bytes);
        }
        m.cv.notify_all();
        std::lock_guard<std::mutex> lk(fake::g_stat_mu);
        ++fake::g_sends;
        return STENCIL_OK;
    }
    static int recv(void* p, size_t bytes, int peer, Comm c, Stream) {
        if (peer < 0 || peer >= c->nranks) return set_error(STENCIL_EINVAL, "fake recv from rank %d of %d", peer, c->nranks);
        {
            std::lock_guard<std::mutex> lk(fake::g_stat_mu);
            ++fake::g_recvs;
        }
        if (fake::t_group > 0) {
            fake::t_pending.push_back({p, bytes, peer, c});
            return STENCIL_OK;
        }
        return fake::take(p, bytes, peer, c);
    }
};

}  // namespace stencil

struct fake_slab_job : stencil::slab::Job<stencil::FakeDev> {};

using stencil::FakeDev;
namespace core = stencil::slab;

extern "C" {

const char* fake_slab_last_error_message(void) { return stencil::g_msg; }
void fake_slab_set_k(int32_t k) { stencil::fake::g_k = k; }
void fake_slab_set_signal(int32_t on) { stencil::fake::g_signal = on != 0; }
void fake_slab_set_free_bytes(int64_t b) { stencil::fake::g_free = b; }
// sweeps, face-signalled sweeps, sends, receives, peer copies since the last reset
void fake_slab_stats(int64_t* out5, int32_t reset) {
    std::lock_guard<std::mutex> lk(stencil::fake::g_stat_mu);
    using namespace stencil::fake;
    if (out5) {
        out5[0] = g_sweeps;
        out5[1] = g_signal_sweeps;
        out5[2] = g_sends;
        out5[3] = g_recvs;
        out5[4] = g_peer_copies;
    }
    if (reset) g_sweeps = g_signal_sweeps = g_sends = g_recvs = g_peer_copies = 0;
}

// gated launches, gate numbering violations, exchange-completion stores since the last reset
void fake_slab_gate_stats(int64_t* out3, int32_t reset) {
    std::lock_guard<std::mutex> lk(stencil::fake::g_stat_mu);
    using namespace stencil::fake;
    if (out3) {
        out3[0] = g_gated;
        out3[1] = g_gate_bad;
        out3[2] = g_xdone;
    }
    if (reset) g_gated = g_gate_bad = g_xdone = 0;
}

int fake_slab_create(const stencil_problem* g, int32_t n, const int32_t* devs, int32_t ex, int32_t flags,
                     fake_slab_job** job) {
    return core::create<FakeDev>(g, n, devs, ex, flags, 0, job);
}
int fake_slab_create2(const stencil_problem* g, int32_t n, const int32_t* devs, int32_t ex, int32_t flags,
                      int64_t margin, fake_slab_job** job) {
    return core::create<FakeDev>(g, n, devs, ex, flags, margin, job);
}
int fake_slab_unique_id(void* id, int64_t bytes) {
    if (!id || bytes < STENCIL_SLAB_ID_BYTES) return stencil::set_error(STENCIL_EINVAL, "id buffer too small");
    std::random_device rd;
    std::memset(id, 0, size_t(STENCIL_SLAB_ID_BYTES));
    std::snprintf(static_cast<char*>(id), size_t(STENCIL_SLAB_ID_BYTES), "rank:%u:%u:%u", rd(), rd(), rd());
    return STENCIL_OK;
}
int fake_slab_create_rank(const stencil_problem* g, int32_t nranks, int32_t rank, int32_t dev, const void* id,
                          int64_t id_bytes, int32_t flags, fake_slab_job** job) {
    return core::create_rank<FakeDev>(g, nranks, rank, dev, id, id_bytes, flags, 0, job);
}
int fake_slab_create_rank2(const stencil_problem* g, int32_t nranks, int32_t rank, int32_t dev, const void* id,
                           int64_t id_bytes, int32_t flags, int64_t margin, fake_slab_job** job) {
    return core::create_rank<FakeDev>(g, nranks, rank, dev, id, id_bytes, flags, margin, job);
}
int fake_slab_destroy(fake_slab_job* job) {
    core::release<FakeDev>(job);
    return STENCIL_OK;
}
int fake_slab_info(const fake_slab_job* job, int32_t slab, int64_t* first, int64_t* planes, int32_t* dev, int32_t* k) {
    return core::info<FakeDev>(job, slab, first, planes, dev, k);
}
int fake_slab_rolling_info(const fake_slab_job* job, int64_t* margin, int64_t* launches) {
    return core::rolling_info<FakeDev>(job, margin, launches);
}
int fake_slab_fill_initial(fake_slab_job* job, int32_t kind, uint64_t seed) {
    return core::fill_initial<FakeDev>(job, kind, seed);
}
int fake_slab_upload(fake_slab_job* job, const void* host, int64_t row, int64_t rows) {
    return core::upload<FakeDev>(job, host, row, rows);
}
int fake_slab_download(fake_slab_job* job, void* host, int64_t row, int64_t rows) {
    return core::download<FakeDev>(job, host, row, rows);
}
int fake_slab_run(fake_slab_job* job, uint32_t iterations, float* ms) { return core::run<FakeDev>(job, iterations, ms); }
int fake_slab_kernel_timing(fake_slab_job* job, int32_t enable) { return core::kernel_timing<FakeDev>(job, enable); }
int fake_slab_kernel_time(fake_slab_job* job, float* ms, int64_t* n, int64_t* cells, int32_t* sig) {
    return core::kernel_time<FakeDev>(job, ms, n, cells, sig);
}
int fake_slab_exchange_time(fake_slab_job* job, float* transfer_ms, float* beside_ms, int64_t* n) {
    return core::exchange_time<FakeDev>(job, transfer_ms, beside_ms, n);
}
int fake_slab_plane_sums(fake_slab_job* job, double* sums) { return core::plane_sums<FakeDev>(job, sums); }
// the fake's layout arithmetic, compared with the product's stencil_layout_init
int fake_slab_layout_init(const stencil_problem* p, stencil_layout* out) { return FakeDev::layout_init(p, out); }
int fake_slab_round_form(const fake_slab_job* job, int32_t* form) { return core::round_form<FakeDev>(job, form); }
int fake_slab_round_info(const fake_slab_job* job, int32_t* form, int32_t* gated, int32_t* confined) {
    return core::round_info<FakeDev>(job, form, gated, confined);
}
int fake_slab_exchange_budget(const fake_slab_job* job, int32_t* cus, int32_t* alt, float* ms, float* alt_ms) {
    return core::exchange_budget<FakeDev>(job, cus, alt, ms, alt_ms);
}
int fake_slab_set_timeout(fake_slab_job* job, int64_t ms) { return core::set_timeout<FakeDev>(job, ms); }

}  // extern "C"
