// sml_hybrid.hip -- the hybrid prediction loop of one rank, native: reservoir predict
// for the rank's regions, the outvec exchange (RCCL all-gather over xGMI), the
// global grid assembly, SPEEDY's run_model on the GPU, and the re-tiling of the
// next step's inputs.
//
// Reference: the time loop of src/parallelmain.f90:204-270 -- `predict` per region
// (:225-234), `sendrecievegrid` (src/mpires.f90:218-780: outvecs gathered at the root
// :338-430, assembled :300-478, `run_model` :549 -> :1516-1628, tiles scattered
// :558-751, `run_speedy` broadcast :721), and the loop exit on run_speedy
// (:268-270).  The startup communicator (startmpi, mpires.f90:21-37) becomes an RCCL
// communicator (sml_comm).
//
// Schedule ("Overlap"): predict needs the feedback tiles for
// the state update and for W_out(:, ncs+1:) x~, and SPEEDY's local vector only for
// W_out(:, 1:ncs) local_model -- the split the reference computes under
// outvec_component_contribs (mod_reservoir.f90:1456-1459).  With overlap on, the
// update + v_ml readout (main stream) run while SPEEDY integrates the previous
// step's window (side stream), on disjoint CUs; results are bit-identical to the
// one-stream schedule.
//
//   main : begin(fb_t) .. wait(lm_t) finish_grid -> [all-gather] -> assemble -> tile fb_t+1
//   side :   [run_model of step t-1 -> forecast grids]            wait(grid_t) run_model ..
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <new>
#include <string>
#include <thread>
#include <cstdlib>
#include <vector>

#include "sml_internal.hpp"
#include "sml_timeline.hpp"

SML_TL_DEFINE(hybrid)

using namespace sml;

struct sml_comm {
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0;
};

struct sml_hybrid {
    sml_reservoirs *res = nullptr;
    sml_dynamics *dyn = nullptr;
    sml_comm *comm = nullptr;
    int numregions = 0, nlocal = 0, ncs = 0, nout = 0;
    int nleap = 24;
    double delt = 900.0, alph = 0.5, rob = 0.05, wil = 0.53;
    bool overlap = true;
    hipStream_t main = nullptr, side = nullptr;
    bool own_streams = false;
    // the two cross-stream dependencies of the overlapped schedule (grid_t: main ->
    // side, lm_t: side -> main): a sequence number in device memory that the
    // producer's stream writes and the consumer's waits for (CP stream memory
    // operations: 3.9 us from the producer's end to the consumer's start on gfx950,
    // 10 us for an event record + wait; tools/probe_hop.hip).  A wait-value packet
    // blocks its queue until the producer's write lands, so under serialised dispatch
    // (rocprofv3 counter passes, AMD_SERIALIZE_KERNEL) it can stall ahead of that
    // producer: SML_HOP_AUTO then takes event hops (sml_hybrid_set_hop_mode).
    // (the chain on SPEEDY's stream, SML_CHAIN_SPEEDY, hops the other way: grid_t,
    // side -> main, before the re-tiling; begun_t, main -> side, before the finish)
    // SML_HOP_KERNEL (the default unless dispatch is serialised): the same sequence
    // numbers, stored by a one-lane kernel behind the producer (k_hop_signal) and
    // polled by the consumer -- inside the v_p finish and run_model's entry specx, which
    // load everything else first, or by a one-lane k_hop_wait elsewhere.  The CP's
    // stream operations run as blit kernels of ~6 us each with a ~6 us boundary in
    // front; measured in an 8-rank share, the chain around the window 45.7 -> 34.8 us
    enum { kHopGrid = 0, kHopLm = 1, kHopBegun = 2, kHops = 3 };
    static constexpr int kSeqStride = 16;  // one 128-B line per hop's word; the late word after them
    hipEvent_t ev[kHops] = {nullptr, nullptr, nullptr};
    uint64_t *d_seq = nullptr, seq[kHops] = {0, 0, 0};
    // a kernel hop that gave up waiting (its consumer read NaN instead of stale data):
    // a pinned host word the waits store at system scope, read without a copy by
    // sml_hybrid_step / run_speedy / sync; the waits' give-up time (wall_clock64 ticks)
    unsigned *h_late = nullptr;
    long long hop_timeout = 400000000ll;
    // where the step's serial chain runs (sml_hybrid_set_chain): false, the two-stream
    // schedule above (the finish, exchange and assembly on the main stream, two hops
    // around every window); true, on SPEEDY's stream right after the window:
    //   side : window_t-1 .. wait(begun_t) finish -> [all-gather] -> assemble -> signal(grid_t) -> window_t
    //   main :   wait(grid_t-1) tile fb_t -> begin_t -> signal(begun_t)        wait(grid_t) tile ..
    // so no hop sits between two pieces of the critical path (the re-tiling and the
    // begin, which need the assembled grid, are the main stream's)
    int chain_mode = SML_CHAIN_AUTO;
    bool chain = false;
    bool use_events = false, use_kernels = false;
    int hop_mode = SML_HOP_AUTO;
    // caller-owned device buffers
    double *fb = nullptr, *lm = nullptr, *ov = nullptr, *g4 = nullptr, *g2 = nullptr, *pr = nullptr, *f4 = nullptr,
           *f2 = nullptr;
    const double *tisr = nullptr;
    // exchange staging (world > 1): send [maxc][nout], recv [world][maxc][nout],
    // and the region-order permutation when the shares are uneven
    int maxc = 0;
    bool contiguous = true;
    double *d_send = nullptr, *d_recv = nullptr, *d_glob = nullptr;
    int32_t *d_perm = nullptr;
    bool started = false, predicted = false, advanced = false;
    // sml_hybrid_step on one rank: the finish also assembled the grids (the exchange is
    // the identity), so the advance that follows skips sml_exchange_assemble
    bool assembled = false;
    // pipelined (sml_hybrid_set_pipelined): each advance issues the next step's begin
    // (update + v_ml readout) on the main stream as soon as its feedback is tiled;
    // begun_next: that begin is in flight, so the next predict only finishes
    bool pipelined = false, begun_next = false;
    // sml_hybrid_set_force_exchange: a world-1 loop with a transport takes the world > 1
    // exchange path (send slab -> ncclAllGather -> advance from the receive slab)
    bool force_exchange = false;
    int64_t allgathers = 0;  // ncclAllGather calls issued by sml_hybrid_step (sml_hybrid_exchanges)
    // get_tisr_by_date (mpires.f90:1644-1676): a table of hourly global tisr fields
    // [nhours][48][96] on the device, the calendar's start year, the hours before the
    // first prediction step and the hours per step; t = steps advanced so far
    const double *tisr_table = nullptr;
    int tisr_nhours = 0, tisr_startyear = 0, tisr_feb29 = 0;
    int64_t tisr_base = 0, tisr_step_hours = 6, t = 0;
    // the window's date (run_model, mpires.f90:1545): with the calendar on
    // (sml_hybrid_set_calendar) every advance hands SPEEDY the date of hour
    // tisr_base + t * tisr_step_hours and the window's forcing follows it (sml_dyn_fordate)
    bool cal_on = false;
    // the exchange row: the outvec (nout), + the slab ocean's sst of the region's
    // resolved points when the slab is on (as sendrecievegrid sends them, mpires.f90:358-383)
    int xw = 0;
    int res_cus = 0;     // the CUs of the main stream's mask (0: no mask)
    int speedy_cus = 0;  // the CUs of the side (SPEEDY) stream's mask (0: no mask)
    // slab ocean (parallelmain.f90:216-249; mpires.f90:288-478, 575-767; cpl_sea.f90:38-46)
    struct Slab {
        sml_reservoirs *res = nullptr;  // the slab reservoirs of this rank's sst regions (generic, ML-only)
        int nslab = 0, nsst = 4, ratio = 28, tot_fb = 0, n_sst_el = 0;
        int timestep = 6, timestep_slab = 168;
        double sst_bias = 0.0;
        const double *base = nullptr, *mask = nullptr;  // base_sst_grid, sea_mask (96, 48)
        double *d_fb = nullptr, *d_ov = nullptr, *d_ring = nullptr, *d_sst = nullptr, *d_ms = nullptr;
        int32_t *d_ring_src = nullptr, *d_row = nullptr, *d_sst_src = nullptr, *d_sfb = nullptr, *d_sgrid = nullptr;
        uint16_t *d_sreg = nullptr;
        bool dirty = false, started = false;
    } slab;
};

namespace {

const char *nccl_msg(ncclResult_t r) { return ncclGetErrorString(r); }

#define SML_NCCL(expr)                                                                                       \
    do {                                                                                                     \
        ncclResult_t r_ = (expr);                                                                            \
        if (r_ != ncclSuccess) return ::sml::fail(SML_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, nccl_msg(r_)); \
    } while (0)

// global region order from the all-gather's [rank][maxc] slabs: glob row r = slab row
// perm[r] (sml_exchange_plan)
__global__ void k_gather_rows(const double *__restrict__ recv, const int32_t *__restrict__ perm,
                              double *__restrict__ glob, int nout, int total) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int r = e / nout, o = e % nout;
    glob[e] = recv[(size_t)perm[r] * nout + o];
}

// ---- slab ocean kernels (mpires.f90:288-478, 575-767)
// the slab feedback: the mean of the ring of the last timestep_slab/timestep - 1 atmo
// feedback subsets, summed column by column as Fortran's sum(.., dim=2) (mpires.f90:757)
__global__ void k_slab_avg(const double *__restrict__ ring, int ncol, int tot, double *__restrict__ fb) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= tot) return;
    double s = 0.0;
    for (int c = 0; c < ncol; ++c) s = s + ring[(size_t)c * tot + e];
    fb[e] = s / (double)ncol;
}

// averaged_atmo_input_vec(:, col) = the atmo feedback at atmo_training_data_idx
// (mpires.f90:755; the index list of trained_ocean_reservoir_prediction,
// mod_slab_ocean_reservoir.f90:1550-1563)
__global__ void k_slab_ring(const double *__restrict__ fb, const int32_t *__restrict__ src, int tot,
                            double *__restrict__ col) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < tot) col[e] = fb[src[e]];
}

// the sst columns of the exchange rows: 272 for a region without a slab prediction
// (mpires.f90:366-372), the slab outvec otherwise
__global__ void k_slab_rows(const double *__restrict__ slab_ov, const int32_t *__restrict__ row, int nslab, int nsst,
                            int nlocal, int nout, int xw, bool fill, double *__restrict__ ov) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (fill) {
        if (e < nlocal * nsst) ov[(size_t)(e / nsst) * xw + nout + e % nsst] = 272.0;
        return;
    }
    if (e < nslab * nsst) ov[(size_t)row[e / nsst] * xw + nout + e % nsst] = slab_ov[e];
}

// wholegrid_sst from every region's sst columns (tile_full_2d_grid_with_local_res,
// res_domain.f90), land / permanent ice to base_sst_grid, floor 272 K
// (mpires.f90:458-472; train_on_sst_anomalies off)
__global__ void k_sst_grid(const double *__restrict__ ov_all, const int32_t *__restrict__ src,
                           const double *__restrict__ base, const double *__restrict__ mask, double *__restrict__ sst) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kGrid2d) return;
    double v = ov_all[src[p]];
    if (mask[p] > 0.0) v = base[p];
    if (v < 272.0) v = 272.0;
    sst[p] = v;
}

// the atmo feedback's sst entries: the overlap tile of wholegrid_sst standardized with
// the slab reservoir's sst mean / std (tile_4d_and_logp_to_local_state_input_slab +
// standardize_data_given_pars1d, mpires.f90:575-581, copied over at :733-736)
__global__ void k_sst_feedback(const double *__restrict__ sst, const int32_t *__restrict__ fbi,
                               const int32_t *__restrict__ gi, const uint16_t *__restrict__ reg,
                               const double *__restrict__ ms, int n, double *__restrict__ fb) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const int j = reg[e];
    const double t = sst[gi[e]] - ms[2 * j];
    fb[fbi[e]] = t / ms[2 * j + 1];
}

}  // namespace

// ------------------------------------------------------------- exchange plan
// The all-gather's layout for `world` ranks of processor_decomposition
// (res_domain.f90:31-62): every rank sends its outvecs zero-padded to the largest
// share maxc, so the receive buffer is [world][maxc][nout]; region r (0-based) sits
// at slab row perm[r] = rank * maxc + (position of r in the rank's list).  With even
// shares (numregions % world == 0) the slabs are already global region order
// (*contiguous = 1); else rank q in 1..left also owns region numregions - left + q - 1
// at the end of its list and k_gather_rows applies perm.  perm may be NULL.
extern "C" int sml_exchange_plan(int numregions, int world, int *maxc, int *contiguous, int32_t *perm) {
    SML_REQUIRE(numregions > 0 && world >= 1 && world <= numregions && maxc && contiguous, "bad argument");
    std::vector<int> all(numregions);
    int mc = 0, c0 = -1;
    bool contig = true;
    for (int r = 0; r < world; ++r) mc = std::max(mc, processor_regions(numregions, world, r, all.data()));
    std::vector<int32_t> p(numregions, -1);
    for (int r = 0; r < world; ++r) {
        const int c = processor_regions(numregions, world, r, all.data());
        if (c0 < 0) c0 = c;
        if (c != c0) contig = false;
        for (int i = 0; i < c; ++i) {
            SML_REQUIRE(p[all[i]] < 0, "region %d owned twice", all[i]);
            p[all[i]] = r * mc + i;
            if (all[i] != r * c0 + i) contig = false;
        }
    }
    for (int r = 0; r < numregions; ++r) SML_REQUIRE(p[r] >= 0, "region %d owned by no rank", r);
    *maxc = mc;
    *contiguous = contig ? 1 : 0;
    if (perm) std::memcpy(perm, p.data(), sizeof(int32_t) * numregions);
    return SML_OK;
}

// ---------------------------------------------------------------- communicator
extern "C" int sml_comm_unique_id(unsigned char *id) {
    SML_REQUIRE(id, "null argument");
    ncclUniqueId u;
    SML_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return SML_OK;
}

extern "C" int sml_comm_create(int world, int rank, const unsigned char *id, sml_comm **out) {
    SML_REQUIRE(out && world >= 1 && rank >= 0 && rank < world && id, "bad argument");
    *out = nullptr;
    sml_comm *c = new (std::nothrow) sml_comm();
    if (!c) return fail(SML_ERR_NOMEM, "host allocation failed");
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(SML_ERR_HIP, "ncclCommInitRank(%d of %d): %s", rank, world, nccl_msg(r));
    }
    c->world = world;
    c->rank = rank;
    *out = c;
    return SML_OK;
}

// rank 0 writes the unique id to `path` (atomically: temp file + rename), the other
// ranks wait for it -- the rendezvous a host without MPI needs
extern "C" int sml_comm_create_file(int world, int rank, const char *path, int timeout_s, sml_comm **out) {
    SML_REQUIRE(out && path && world >= 1 && rank >= 0 && rank < world, "bad argument");
    unsigned char id[NCCL_UNIQUE_ID_BYTES];
    if (rank == 0) {
        if (int rc = sml_comm_unique_id(id)) return rc;
        std::string tmp = std::string(path) + ".tmp";
        FILE *f = std::fopen(tmp.c_str(), "wb");
        if (!f) return fail(SML_ERR_IO, "cannot write %s", tmp.c_str());
        const size_t w = std::fwrite(id, 1, sizeof id, f);
        std::fclose(f);
        if (w != sizeof id || std::rename(tmp.c_str(), path) != 0) return fail(SML_ERR_IO, "cannot publish %s", path);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            FILE *f = std::fopen(path, "rb");
            if (f) {
                const size_t r = std::fread(id, 1, sizeof id, f);
                std::fclose(f);
                if (r == sizeof id) break;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s > 0 ? timeout_s : 60))
                return fail(SML_ERR_IO, "timed out waiting for %s", path);
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
    }
    return sml_comm_create(world, rank, id, out);
}

// a rank descriptor without a transport: world and rank for sml_hybrid_create when
// the host moves the outvec slabs itself (sml_hybrid_advance_slabs)
extern "C" int sml_comm_create_local(int world, int rank, sml_comm **out) {
    SML_REQUIRE(out && world >= 1 && rank >= 0 && rank < world, "bad argument");
    *out = nullptr;
    sml_comm *c = new (std::nothrow) sml_comm();
    if (!c) return fail(SML_ERR_NOMEM, "host allocation failed");
    c->world = world;
    c->rank = rank;
    *out = c;
    return SML_OK;
}

extern "C" int sml_comm_destroy(sml_comm *c) {
    if (!c) return SML_OK;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
    return SML_OK;
}

extern "C" int sml_comm_rank(const sml_comm *c, int *world, int *rank) {
    SML_REQUIRE(c, "null communicator");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    return SML_OK;
}

extern "C" int sml_comm_allgather(sml_comm *c, const double *d_send, double *d_recv, int64_t count, void *stream) {
    SML_REQUIRE(c && d_send && d_recv && count >= 0, "bad argument");
    if (!c->comm) return fail(SML_ERR_STATE, "rank %d of %d is a local descriptor without a transport", c->rank, c->world);
    SML_NCCL(ncclAllGather(d_send, d_recv, (size_t)count, ncclDouble, c->comm, (hipStream_t)stream));
    return SML_OK;
}

// ------------------------------------------------------------------ calendar
// The reference's calendar arithmetic (src/mod_calendar.f90), restated with its
// quirks: get_current_time_delta_hour (:24-92) counts years of 8760 h from the
// start year (start month / day / hour unused), subtracts the leap days of the
// elapsed years, walks a 365-day month table whose February it sets to 29 in a leap
// year -- the table is a SAVEd local, so once a leap year is met February keeps 29
// days for the rest of the run (*feb29 carries that state) -- and an exact month
// boundary falls to December 31 of the year before; numof_hours_into_year
// (:133-175) counts whole months, days, the hour, and 0 -> 1.  get_tisr_by_date
// (mpires.f90:1665-1671) then wraps indices past 8760 by 8760.
namespace {
bool leap_year(int y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }  // leap_year_check :94-106
}  // namespace

// get_current_time_delta_hour (mod_calendar.f90:24-92): date[4] = currentyear,
// currentmonth, currentday, currenthour after hours_elapsed hours from startyear
extern "C" int sml_calendar_delta_hour(int startyear, int64_t hours_elapsed, int *feb29, int *date) {
    SML_REQUIRE(feb29 && date && hours_elapsed >= 0, "bad argument");
    const int64_t hours_in_year = 8760, hours_in_a_day = 24;
    const int64_t years = hours_elapsed / hours_in_year;
    int year = (int)(years + startyear);
    int leap_days = 0;
    for (int64_t i = 0; i < years; ++i)
        if (leap_year(startyear + (int)i)) ++leap_days;
    if (leap_year(year)) *feb29 = 1;
    const int ncal[12] = {31, *feb29 ? 29 : 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    const int64_t day_of_year = (hours_elapsed % hours_in_year) / hours_in_a_day - leap_days;
    int64_t counter = day_of_year;
    int month = 1;
    while (counter > 0) {
        counter -= ncal[month - 1];
        ++month;
    }
    month -= 1;
    if (month <= 0) {
        month = 12;
        year -= 1;
    }
    date[0] = year;
    date[1] = month;
    date[2] = (int)(ncal[month - 1] + counter);
    date[3] = (int)(hours_elapsed % hours_in_a_day);
    return SML_OK;
}

extern "C" int sml_tisr_date_index(int startyear, int64_t hours_elapsed, int *feb29, int *index) {
    SML_REQUIRE(feb29 && index && hours_elapsed >= 0, "bad argument");
    int d[4];
    if (int rc = sml_calendar_delta_hour(startyear, hours_elapsed, feb29, d)) return rc;
    const int year = d[0], month = d[1], day = d[2], hour = d[3];
    // numof_hours_into_year(year, month, day, hour) with the year's own leap table
    const bool ly = leap_year(year);
    const int nmon[12] = {31, ly ? 29 : 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    int64_t n = 0;
    for (int i = 1; i < month; ++i) n += 24 * nmon[i - 1];
    for (int i = 1; i < day; ++i) n += 24;
    n += hour;
    if (n == 0) n = 1;
    if (n > 24 * 365) n -= 24 * 365;
    *index = (int)n;
    return SML_OK;
}

// ------------------------------------------------------------------ hybrid loop
namespace {

// SML_HOP_KERNEL's two kernels.  The producer's data is released by its own kernel's
// end (the dispatch after it on the same stream starts behind that release), so the
// signal is one relaxed agent-scope store of the sequence number (a vector store,
// write-through: MI355X_MICROARCH.md inter-workgroup visibility), and the consumer's
// next dispatch acquires at its start like any kernel's.  The wait polls with relaxed
// agent loads and s_sleep from one lane; it never spins forever: after ~4 s it marks
// the late word (sml_hybrid_sync reports it) and lets the stream go on.
__global__ void k_hop_signal(uint64_t *flag, uint64_t v) {
    SML_TL_SCOPE(sml::tl::kHopSignal);
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_hop_wait(const uint64_t *flag, uint64_t v, unsigned *late, long long timeout) {
    if (threadIdx.x != 0) return;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > timeout) {  // default ~4 s at wall_clock64's 100 MHz
            __hip_atomic_store(late, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
    }
}

unsigned *hop_late_word(sml_hybrid *h) { return h->h_late; }

// a hop that timed out since the last report: SML_ERR_STATE once (the word is reset)
int hop_late_check(sml_hybrid *h, const char *where) {
    if (h->h_late && __atomic_load_n(h->h_late, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(h->h_late, 0u, __ATOMIC_RELEASE);
        return fail(SML_ERR_STATE, "%s: a cross-stream hop (SML_HOP_KERNEL) timed out -- its consumer read NaN, "
                                   "the steps since are invalid", where);
    }
    return SML_OK;
}

// producer side of hop `k`: ordered after everything issued on `s` so far
int hop_signal(sml_hybrid *h, int k, hipStream_t s) {
    uint64_t *w = h->d_seq + k * sml_hybrid::kSeqStride;
    if (h->use_events) {
        SML_HIP(hipEventRecord(h->ev[k], s));
    } else if (h->use_kernels) {
        hipLaunchKernelGGL(k_hop_signal, dim3(1), dim3(64), 0, s, w, ++h->seq[k]);
        SML_HIP(hipGetLastError());
    } else {
        SML_HIP(hipStreamWriteValue64(s, w, ++h->seq[k], 0));
    }
    return SML_OK;
}

// consumer side: `s` waits for the latest signal of hop `k`
int hop_wait(sml_hybrid *h, int k, hipStream_t s) {
    uint64_t *w = h->d_seq + k * sml_hybrid::kSeqStride;
    if (h->use_events) {
        SML_HIP(hipStreamWaitEvent(s, h->ev[k], 0));
    } else if (h->use_kernels) {
        hipLaunchKernelGGL(k_hop_wait, dim3(1), dim3(64), 0, s, w, h->seq[k], hop_late_word(h), h->hop_timeout);
        SML_HIP(hipGetLastError());
    } else {
        SML_HIP(hipStreamWaitValue64(s, w, h->seq[k], hipStreamWaitValueGte, ~0ull));
    }
    return SML_OK;
}

// the exchange staging for rows of h->xw doubles (world > 1): the loop's own
// all-gather's send / receive slabs (when the communicator has a transport) and the
// region-order copy of uneven shares
int alloc_exchange(sml_hybrid *h) {
    for (double **p : {&h->d_send, &h->d_recv, &h->d_glob})
        if (*p) {
            (void)hipFree(*p);
            *p = nullptr;
        }
    const size_t row = (size_t)h->xw * 8;
    const int world = h->comm->world;
    if (h->comm->comm && h->maxc > 0 &&
        (hipMalloc(&h->d_send, (size_t)h->maxc * row) != hipSuccess ||
         hipMalloc(&h->d_recv, (size_t)world * h->maxc * row) != hipSuccess ||
         hipMemset(h->d_send, 0, (size_t)h->maxc * row) != hipSuccess))
        return fail(SML_ERR_NOMEM, "exchange buffers");
    if (!h->contiguous && hipMalloc(&h->d_glob, (size_t)h->numregions * row) != hipSuccess)
        return fail(SML_ERR_NOMEM, "exchange buffers");
    return SML_OK;
}

// dispatch serialised by the runtime or a profiler: the HIP runtime's
// AMD_SERIALIZE_KERNEL, rocprofv3's counter collection (ROCPROF_COUNTER_COLLECTION,
// set by `rocprofv3 --pmc` / `-i`)
bool env_on(const char *name) {
    const char *e = getenv(name);
    return e && *e && std::strcmp(e, "0") != 0 && std::strcmp(e, "false") != 0 && std::strcmp(e, "False") != 0;
}

bool dispatch_serialised() { return env_on("AMD_SERIALIZE_KERNEL") || env_on("ROCPROF_COUNTER_COLLECTION"); }

}  // namespace

// hop mode: SML_HOP_AUTO (kernel hops on CU-disjoint streams, event hops when dispatch
// is serialised or SML_HYBRID_EVENTS=1, wait-value hops otherwise), SML_HOP_WAIT_VALUE,
// SML_HOP_EVENTS, SML_HOP_KERNEL.  Both streams are drained first, so no wait of one
// kind is left pending on a signal of the other.
extern "C" int sml_hybrid_set_hop_mode(sml_hybrid *h, int mode) {
    SML_REQUIRE(h && (mode == SML_HOP_AUTO || mode == SML_HOP_WAIT_VALUE || mode == SML_HOP_EVENTS ||
                      mode == SML_HOP_KERNEL),
                "bad hop mode %d", mode);
    if (h->main) SML_HIP(hipStreamSynchronize(h->main));
    if (h->side && h->side != h->main) SML_HIP(hipStreamSynchronize(h->side));
    h->hop_mode = mode;
    if (mode == SML_HOP_AUTO) {
        // kernel hops only when the two streams run on disjoint CUs (res_cus > 0): a
        // waiting finish's blocks then never occupy a CU the window (their producer)
        // needs; not when dispatch is serialised (a waiting kernel would hold its queue
        // ahead of its producer) or SML_HYBRID_EVENTS=1 asks for event hops (the PMC
        // passes of profiles/collect.sh)
        h->use_events = env_on("SML_HYBRID_EVENTS") || dispatch_serialised();
        h->use_kernels = !h->use_events && h->res_cus > 0;
    } else {
        h->use_events = mode == SML_HOP_EVENTS;
        h->use_kernels = mode == SML_HOP_KERNEL;
    }
    return SML_OK;
}

// the give-up time of every in-kernel wait of the loop (the kernel hops, and run_model's
// exit waiting for its safety check), microseconds; default 4 s (hops) / 1 s (check)
extern "C" int sml_hybrid_set_hop_timeout(sml_hybrid *h, int64_t microseconds) {
    SML_REQUIRE(h && microseconds >= 0, "bad argument");
    if (h->main) SML_HIP(hipStreamSynchronize(h->main));
    if (h->side && h->side != h->main) SML_HIP(hipStreamSynchronize(h->side));
    h->hop_timeout = (long long)microseconds * 100;  // wall_clock64 runs at 100 MHz
    return sml::dyn_set_check_timeout(h->dyn, std::min<long long>(h->hop_timeout, 100000000ll));
}

// pipelined loop (see sml_hybrid::pipelined); switching it off keeps a begin already
// in flight for the next predict
extern "C" int sml_hybrid_set_pipelined(sml_hybrid *h, int on) {
    SML_REQUIRE(h, "null context");
    h->pipelined = on != 0;
    return SML_OK;
}

// the step's serial chain (finish -> exchange -> assembly -> tiling): on the main
// stream between two cross-stream hops (SML_CHAIN_TWO_STREAMS), or on SPEEDY's stream
// right after the window (SML_CHAIN_SPEEDY).  SML_CHAIN_AUTO is the two-stream form:
// measured same-box (r04a), the chain on SPEEDY's stream was 19-20 us per step SLOWER
// at world 1 and in the 8-rank share -- its two remaining stream operations
// (hipStreamWaitValue64 / WriteValue64 run as blit kernels, ~6 us each, satisfied or
// not) stay on the critical path, and the finish and assembly get 64 CUs instead of
// 192.  With kernel hops it has no hop kernel on SPEEDY's stream at all (the finish
// waits for its begin in-kernel, the entry specx signals the grid) and still loses
// (r04, profiles/r04/chain_nohop: N = 1 1104 / 1109 vs 1123 / 1123 steps/s, 8-rank
// share 1185 / 1186 vs 1194 / 1195): the finish and assembly on 64 CUs cost more than
// the two signal kernels.  Drains both streams first.
extern "C" int sml_hybrid_set_chain(sml_hybrid *h, int mode) {
    SML_REQUIRE(h && (mode == SML_CHAIN_AUTO || mode == SML_CHAIN_TWO_STREAMS || mode == SML_CHAIN_SPEEDY),
                "bad chain mode %d", mode);
    SML_REQUIRE(!h->predicted, "sml_hybrid_set_chain between predict and advance");
    if (h->main) SML_HIP(hipStreamSynchronize(h->main));
    if (h->side && h->side != h->main) SML_HIP(hipStreamSynchronize(h->side));
    h->chain_mode = mode;
    h->chain = mode == SML_CHAIN_SPEEDY && h->overlap && h->side != h->main;
    return SML_OK;
}

extern "C" int sml_hybrid_chain(const sml_hybrid *h, int *requested, int *effective) {
    SML_REQUIRE(h, "null context");
    if (requested) *requested = h->chain_mode;
    if (effective) *effective = h->chain ? SML_CHAIN_SPEEDY : SML_CHAIN_TWO_STREAMS;
    return SML_OK;
}

// the stream the local outvecs are ready on after sml_hybrid_predict, and on which a
// host-driven exchange should run before sml_hybrid_advance
extern "C" int sml_hybrid_exchange_stream(const sml_hybrid *h, void **stream) {
    SML_REQUIRE(h && stream, "null argument");
    *stream = h->chain ? h->side : h->main;
    return SML_OK;
}

extern "C" int sml_hybrid_set_force_exchange(sml_hybrid *h, int on) {
    SML_REQUIRE(h, "null context");
    if (on && !h->force_exchange) {
        SML_REQUIRE(h->comm && h->comm->comm, "forcing the exchange needs a communicator with a transport");
        SML_REQUIRE(!h->predicted, "sml_hybrid_set_force_exchange between predict and advance");
        if (h->comm->world == 1) {  // the one-rank plan: maxc = every region, contiguous
            h->maxc = h->nlocal;
            h->contiguous = true;
            if (int rc = alloc_exchange(h)) return rc;
        }
    }
    h->force_exchange = on != 0;
    return SML_OK;
}

// the requested mode and the one in effect (SML_HOP_WAIT_VALUE or SML_HOP_EVENTS)
extern "C" int sml_hybrid_hop_mode(const sml_hybrid *h, int *requested, int *effective) {
    SML_REQUIRE(h, "null context");
    if (requested) *requested = h->hop_mode;
    if (effective) *effective = h->use_events ? SML_HOP_EVENTS : h->use_kernels ? SML_HOP_KERNEL : SML_HOP_WAIT_VALUE;
    return SML_OK;
}

extern "C" int sml_hybrid_destroy(sml_hybrid *h) {
    if (!h) return SML_OK;
    if (h->main) (void)hipStreamSynchronize(h->main);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->own_streams) {
        if (h->side && h->side != h->main) (void)hipStreamDestroy(h->side);
        if (h->main) (void)hipStreamDestroy(h->main);
    }
    for (hipEvent_t e : h->ev)
        if (e) (void)hipEventDestroy(e);
    sml_hybrid::Slab &sl = h->slab;
    void *ptrs[] = {h->d_send, h->d_recv, h->d_glob, h->d_perm, h->d_seq, sl.d_fb, sl.d_ov, sl.d_ring, sl.d_sst, sl.d_ms,
                    sl.d_ring_src, sl.d_row, sl.d_sst_src, sl.d_sfb, sl.d_sgrid, sl.d_sreg};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (h->h_late) (void)hipHostFree(h->h_late);
    delete h;
    return SML_OK;
}

extern "C" int sml_hybrid_create(sml_reservoirs *res, sml_dynamics *dyn, sml_comm *comm, int nleap, double delt,
                                 double alph, double rob, double wil, int overlap, int speedy_cus, sml_hybrid **out) {
    SML_REQUIRE(out && res && dyn && nleap >= 0 && delt > 0.0, "bad argument");
    *out = nullptr;
    sml_hybrid *h = new (std::nothrow) sml_hybrid();
    if (!h) return fail(SML_ERR_NOMEM, "host allocation failed");
    auto bail = [&](int rc) {
        sml_hybrid_destroy(h);
        return rc;
    };
    h->res = res;
    h->dyn = dyn;
    h->comm = comm;
    h->nleap = nleap;
    h->delt = delt;
    h->alph = alph;
    h->rob = rob;
    h->wil = wil;
    h->overlap = overlap != 0;
    if (int rc = sml_res_info(res, &h->numregions, &h->nlocal, &h->ncs, &h->nout, nullptr)) return bail(rc);
    const int world = comm ? comm->world : 1, rank = comm ? comm->rank : 0;
    // the communicator's decomposition must be the one the reservoir context holds
    std::vector<int> mine(h->numregions), ids(h->nlocal);
    const int cnt = processor_regions(h->numregions, world, rank, mine.data());
    if (int rc = sml_res_info(res, nullptr, nullptr, nullptr, nullptr, ids.data())) return bail(rc);
    // (without a communicator any subset is accepted for predict / advance around a
    // host exchange; sml_hybrid_step then needs every region local)
    if (comm && (cnt != h->nlocal || !std::equal(ids.begin(), ids.end(), mine.begin())))
        return bail(fail(SML_ERR_ARG, "the reservoir context does not hold rank %d of %d's processor_decomposition",
                         rank, world));
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return bail(fail(SML_ERR_HIP, "no device"));
    // streams: non-default (the legacy NULL stream would serialise the two chains);
    // with overlap and 0 < speedy_cus < CUs, SPEEDY's chain gets CUs [0, speedy_cus)
    // and the reservoir a disjoint range after it (sml_stream_create_cu_range)
    h->own_streams = true;
    if (h->overlap && speedy_cus > 0 && speedy_cus < ncu) {
        void *s = nullptr, *m = nullptr;
        if (int rc = sml_stream_create_cu_range(0, speedy_cus, &s)) return bail(rc);
        h->side = (hipStream_t)s;
        // the reservoir on CUs [speedy_cus, speedy_cus + res_cus): one CU per 6 of the
        // rank's regions (a multiple of 8: the same count on every XCD), at least 64, at
        // most all the CUs SPEEDY does not use.  At 6 regions per CU the begin (update +
        // v_ml readout) takes about the window's time beside it; more CUs only add HBM
        // pressure on the window, fewer make the begin the critical path.  Same box
        // (DESIGN.md §4): N = 1 (1152 regions) 192 CUs 1137 vs 160 1095; the 2-rank share
        // 96 CUs 1254 vs 192 1230; 4-rank 64 1282 vs 192 1264; 8-rank 64 1298 vs 192
        // 1290 steps/s.  SML_RES_CUS overrides the count.
        int res_cus = std::min(ncu - speedy_cus, std::max(64, ((h->nlocal + 5) / 6 + 7) / 8 * 8));
        if (const char *er = getenv("SML_RES_CUS")) res_cus = std::min(std::max(atoi(er), 1), ncu - speedy_cus);
        if (int rc = sml_stream_create_cu_range(speedy_cus, res_cus, &m)) return bail(rc);
        h->main = (hipStream_t)m;
        // run_model's safety check (re-grid + min/max beside the window) on the CUs
        // left over, else on the reservoir's: never on SPEEDY's, where its blocks
        // slowed the window's first kernels (k_st_gridspec 21 vs 17.6 us, rocprof r02u)
        const int spare = ncu - speedy_cus - res_cus;
        if (int rc = spare > 0 ? sml_dyn_set_check_cus(dyn, speedy_cus + res_cus, spare)
                               : sml_dyn_set_check_cus(dyn, speedy_cus, res_cus))
            return bail(rc);
        if (int rc = sml_res_set_read_waves(res, 0)) return bail(rc);  // pacing pays only on shared CUs
        if (int rc = sml_res_set_update_cus(res, res_cus)) return bail(rc);  // one balanced-update block per CU
        h->res_cus = res_cus;
        h->speedy_cus = speedy_cus;
    } else {
        if (hipStreamCreateWithFlags(&h->main, hipStreamNonBlocking) != hipSuccess)
            return bail(fail(SML_ERR_HIP, "stream"));
        if (h->overlap) {
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            if (hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, hi) != hipSuccess)
                return bail(fail(SML_ERR_HIP, "stream"));
        } else {
            h->side = h->main;
        }
    }
    for (hipEvent_t &e : h->ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return bail(fail(SML_ERR_HIP, "event"));
    if (int rc = sml_hybrid_set_hop_mode(h, SML_HOP_AUTO)) return bail(rc);
    constexpr size_t seq_bytes = sml_hybrid::kHops * sml_hybrid::kSeqStride * sizeof(uint64_t);
    if (hipMalloc(&h->d_seq, seq_bytes) != hipSuccess || hipMemset(h->d_seq, 0, seq_bytes) != hipSuccess ||
        hipHostMalloc((void **)&h->h_late, sizeof(unsigned), hipHostMallocCoherent) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
        return bail(fail(SML_ERR_HIP, "sequence counters"));
    *h->h_late = 0;
    h->xw = h->nout;
    if (world > 1) {
        std::vector<int32_t> perm(h->numregions);
        int contig = 1;
        if (int rc = sml_exchange_plan(h->numregions, world, &h->maxc, &contig, perm.data())) return bail(rc);
        h->contiguous = contig != 0;
        if (!h->contiguous &&
            (hipMalloc(&h->d_perm, (size_t)h->numregions * 4) != hipSuccess ||
             hipMemcpy(h->d_perm, perm.data(), perm.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
            return bail(fail(SML_ERR_NOMEM, "exchange buffers"));
        if (int rc = alloc_exchange(h)) return bail(rc);
    }
    if (int rc = sml_hybrid_set_chain(h, SML_CHAIN_AUTO)) return bail(rc);
    *out = h;
    return SML_OK;
}

extern "C" int sml_hybrid_set_buffers(sml_hybrid *h, double *d_feedback, double *d_local_model, double *d_outvec,
                                      double *d_grid4d, double *d_grid2d, double *d_precip, double *d_fc4d,
                                      double *d_fc2d, const double *d_tisr) {
    SML_REQUIRE(h && d_feedback && d_outvec && d_grid4d && d_grid2d && d_precip && d_fc4d && d_fc2d,
                "null buffer");
    SML_REQUIRE(h->ncs == 0 || d_local_model, "a hybrid context needs d_local_model");
    h->fb = d_feedback;
    h->lm = d_local_model;
    h->ov = d_outvec;
    h->g4 = d_grid4d;
    h->g2 = d_grid2d;
    h->pr = d_precip;
    h->f4 = d_fc4d;
    h->f2 = d_fc2d;
    h->tisr = d_tisr;
    return SML_OK;
}

extern "C" int sml_hybrid_set_tisr(sml_hybrid *h, const double *d_tisr) {
    SML_REQUIRE(h, "null context");
    h->tisr = d_tisr;
    return SML_OK;
}

// the loop's calendar (run_model / get_tisr_by_date's get_current_time_delta_hour,
// mpires.f90:1545, :1661): start year, the hours before the first prediction step
// (traininglength + prediction marker + synclength) and the hours per step; turns on
// the window's date-driven forcing.  Resets the step count and the February latch.
extern "C" int sml_hybrid_set_calendar(sml_hybrid *h, int startyear, int64_t hours_base, int step_hours) {
    SML_REQUIRE(h && step_hours > 0 && hours_base >= 0, "bad argument");
    h->tisr_startyear = startyear;
    h->tisr_base = hours_base;
    h->tisr_step_hours = step_hours;
    h->tisr_feb29 = 0;
    h->t = 0;
    h->cal_on = true;
    return SML_OK;
}

// the calendar date of the next window (the advance after the last one issued)
extern "C" int sml_hybrid_window_date(sml_hybrid *h, int *date) {
    SML_REQUIRE(h && date, "null argument");
    SML_REQUIRE(h->cal_on, "no calendar (sml_hybrid_set_calendar)");
    int feb29 = h->tisr_feb29;
    return sml_calendar_delta_hour(h->tisr_startyear, h->tisr_base + (h->t + 1) * h->tisr_step_hours, &feb29, date);
}

extern "C" int sml_hybrid_set_tisr_table(sml_hybrid *h, const double *d_table, int nhours, int startyear,
                                         int64_t hours_base, int step_hours) {
    SML_REQUIRE(h && (d_table == nullptr || (nhours >= 8760 && step_hours > 0 && hours_base >= 0)), "bad argument");
    h->tisr_table = d_table;
    h->tisr_nhours = nhours;
    h->tisr_startyear = startyear;
    h->tisr_base = hours_base;
    h->tisr_step_hours = step_hours;
    h->tisr_feb29 = 0;
    h->t = 0;
    return SML_OK;
}

// the SAVEd February of the reference's month table (mod_calendar.f90:40,61-63) as
// the host's own calendar calls left it: every get_current_time_delta_hour of the
// process shares it (training windows mod_reservoir.f90:355/632/638, the prediction
// start mpires.f90:108/489, run_model :1545), so a host that met a leap year before
// the loop's first tisr lookup passes 1 here.  sml_hybrid_set_tisr_table resets it
// to 0 (a process whose calendar has not met a leap year).
extern "C" int sml_hybrid_set_feb29(sml_hybrid *h, int feb29) {
    SML_REQUIRE(h, "null context");
    h->tisr_feb29 = feb29 != 0;
    return SML_OK;
}

extern "C" int sml_hybrid_get_feb29(const sml_hybrid *h, int *feb29) {
    SML_REQUIRE(h && feb29, "null argument");
    *feb29 = h->tisr_feb29;
    return SML_OK;
}

extern "C" int sml_hybrid_streams(const sml_hybrid *h, void **main, void **side) {
    SML_REQUIRE(h, "null context");
    if (main) *main = h->main;
    if (side) *side = h->side;
    return SML_OK;
}

extern "C" int sml_hybrid_cus(const sml_hybrid *h, int *speedy_cus, int *res_cus) {
    SML_REQUIRE(h, "null context");
    if (speedy_cus) *speedy_cus = h->speedy_cus;
    if (res_cus) *res_cus = h->res_cus;
    return SML_OK;
}

// start_prediction's hand-over (src/mod_reservoir.f90:938-959, parallelmain.f90:207-216):
// the first step's feedback tiles from an analysis grid and the local model from a
// SPEEDY forecast of it, both copied into the loop's buffers (on the main stream,
// ordered after the caller's legacy-stream work)
extern "C" int sml_hybrid_start(sml_hybrid *h, const double *d_g4, const double *d_g2, const double *d_pr,
                                const double *d_f4, const double *d_f2) {
    SML_REQUIRE(h && h->fb, "sml_hybrid_set_buffers first");
    SML_REQUIRE(d_g4 && d_g2 && d_pr && d_f4 && d_f2, "null argument");
    SML_HIP(hipDeviceSynchronize());
    // a restart after a pipelined run: the begin the last advance issued was built from
    // the old feedback -- discard it (the state rolls back to the one it read), so the
    // first predict begins from the feedback tiled here
    if (h->begun_next) {
        if (int rc = sml_res_step_cancel(h->res)) return rc;
        h->begun_next = false;
    }
    const size_t n4 = (size_t)kGrid4d * 8, n2 = (size_t)kGrid2d * 8;
    if (d_g4 != h->g4) SML_HIP(hipMemcpyAsync(h->g4, d_g4, n4, hipMemcpyDeviceToDevice, h->main));
    if (d_g2 != h->g2) SML_HIP(hipMemcpyAsync(h->g2, d_g2, n2, hipMemcpyDeviceToDevice, h->main));
    if (d_pr != h->pr) SML_HIP(hipMemcpyAsync(h->pr, d_pr, n2, hipMemcpyDeviceToDevice, h->main));
    if (d_f4 != h->f4) SML_HIP(hipMemcpyAsync(h->f4, d_f4, n4, hipMemcpyDeviceToDevice, h->main));
    if (d_f2 != h->f2) SML_HIP(hipMemcpyAsync(h->f2, d_f2, n2, hipMemcpyDeviceToDevice, h->main));
    if (int rc = sml_res_tile_inputs(h->res, h->g4, h->g2, h->pr, h->f4, h->f2, h->tisr, h->fb, h->lm, h->main))
        return rc;
    if (int rc = hop_signal(h, sml_hybrid::kHopLm, h->main)) return rc;
    SML_HIP(hipStreamSynchronize(h->main));  // (the chain on SPEEDY's stream reads these on the other stream)
    h->started = true;
    h->predicted = h->advanced = false;
    return SML_OK;
}

// ------------------------------------------------------------------ slab ocean
namespace {

// predict_slab_ml for every slab reservoir of the rank on a slab step
// (parallelmain.f90:236-249: mod(t*timestep, timestep_slab) == 0, the default
// ml_only_ocean set by initialize_slab_ocean_model): the feedback is the mean of the
// ring as the previous step's sendrecievegrid left it (mpires.f90:757), and the new
// sst goes into the exchange rows
int slab_predict(sml_hybrid *h) {
    sml_hybrid::Slab &sl = h->slab;
    if (!sl.res) return SML_OK;
    if (!sl.started) return fail(SML_ERR_STATE, "sml_hybrid_start_slab first");
    const int64_t tt = h->t + 1;
    if ((tt * sl.timestep) % sl.timestep_slab != 0) return SML_OK;
    // a slab step on every rank: the other ranks' rows carry new sst, so wholegrid_sst
    // and the window's sst are rebuilt here too, even when this rank predicts none
    sl.dirty = true;
    if (sl.nslab == 0) return SML_OK;
    hipStream_t m = h->main;
    hipLaunchKernelGGL(k_slab_avg, dim3((sl.tot_fb + 255) / 256), dim3(256), 0, m, sl.d_ring, sl.ratio - 1, sl.tot_fb,
                       sl.d_fb);
    SML_HIP(hipGetLastError());
    if (int rc = sml_res_step(sl.res, sl.d_fb, nullptr, sl.d_ov, m)) return rc;
    const int n = sl.nslab * sl.nsst;
    hipLaunchKernelGGL(k_slab_rows, dim3((n + 255) / 256), dim3(256), 0, m, sl.d_ov, sl.d_row, sl.nslab, sl.nsst,
                       h->nlocal, h->nout, h->xw, false, h->ov);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

// sendrecievegrid's sst half (mpires.f90:288-319, 458-472, 575-581, 733-736) after a
// change of any region's slab sst: wholegrid_sst from the exchange rows, the atmo
// feedback's sst entries, and run_model's sst_hybrid into the window (cpl_sea.f90:38-46)
int slab_sst(sml_hybrid *h, const double *d_all, hipStream_t m) {
    sml_hybrid::Slab &sl = h->slab;
    if (!sl.res || !sl.dirty) return SML_OK;
    hipLaunchKernelGGL(k_sst_grid, dim3((kGrid2d + 255) / 256), dim3(256), 0, m, d_all, sl.d_sst_src, sl.base, sl.mask,
                       sl.d_sst);
    SML_HIP(hipGetLastError());
    if (sl.n_sst_el) {
        hipLaunchKernelGGL(k_sst_feedback, dim3((sl.n_sst_el + 255) / 256), dim3(256), 0, m, sl.d_sst, sl.d_sfb,
                           sl.d_sgrid, sl.d_sreg, sl.d_ms, sl.n_sst_el, h->fb);
        SML_HIP(hipGetLastError());
    }
    if (int rc = sml_dyn_set_hybrid_sst(h->dyn, sl.d_sst, sl.sst_bias, m)) return rc;
    sl.dirty = false;
    return SML_OK;
}

template <typename T>
int upload(T **d, const std::vector<T> &v) {
    if (hipMalloc(d, std::max<size_t>(v.size(), 1) * sizeof(T)) != hipSuccess) return fail(SML_ERR_NOMEM, "slab tables");
    if (!v.empty()) SML_HIP(hipMemcpy(*d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return SML_OK;
}

}  // namespace

// the slab ocean in the loop (parallelmain.f90:216-249, sendrecievegrid's sst half).
// Before sml_hybrid_set_buffers: the exchange rows widen to nout + resx*resy.
extern "C" int sml_hybrid_set_slab(sml_hybrid *h, sml_reservoirs *slab, const double *d_base_sst,
                                   const double *d_sea_mask, int timestep, int timestep_slab, double sst_bias) {
    SML_REQUIRE(h && slab && d_base_sst && d_sea_mask, "null argument");
    SML_REQUIRE(!h->slab.res, "the slab ocean is set already");
    SML_REQUIRE(!h->ov, "sml_hybrid_set_slab must precede sml_hybrid_set_buffers (the exchange rows widen)");
    SML_REQUIRE(timestep > 0 && timestep_slab % timestep == 0 && timestep_slab / timestep >= 2,
                "timestep_slab (%d) must be a multiple >= 2 of timestep (%d)", timestep_slab, timestep);
    int snum = 0, nslab = 0, sncs = 0, snout = 0;
    if (int rc = sml_res_info(slab, &snum, &nslab, &sncs, &snout, nullptr)) return rc;
    SML_REQUIRE(snum == h->numregions && sncs == 0, "the slab context must be ML-only (chunk_speedy 0) over the "
                "same %d regions", h->numregions);
    RegionGeom g0;
    SML_REQUIRE(region_geom(h->numregions, 0, &g0) && snout == g0.resx * g0.resy,
                "the slab reservoirs predict the sst of the region's %d points, not %d", g0.resx * g0.resy, snout);
    std::vector<int> ids(h->nlocal), sids(nslab);
    std::vector<int64_t> off(h->nlocal + 1), soff(nslab + 1);
    if (int rc = sml_res_info(h->res, nullptr, nullptr, nullptr, nullptr, ids.data())) return rc;
    if (int rc = sml_res_info(slab, nullptr, nullptr, nullptr, nullptr, sids.data())) return rc;
    if (int rc = sml_res_feedback_offsets(h->res, off.data())) return rc;
    if (int rc = sml_res_feedback_offsets(slab, soff.data())) return rc;
    // the slab reservoirs are those of the rank's regions with an sst input, in order
    // (trained_ocean_reservoir_prediction: sst_bool_prediction <=> sst input)
    std::vector<int32_t> ring_src, row, sfb, sgrid;
    std::vector<uint16_t> sreg;
    int j = 0;
    for (int i = 0; i < h->nlocal; ++i) {
        RegionGeom g;
        region_geom(h->numregions, ids[i], &g);
        const int in2d = g.inx * g.iny, natmo = kVars * in2d * kZGrid;
        int ninp = 0;
        if (int rc = sml_res_ninp(h->res, i, &ninp)) return rc;
        const bool sst = ninp == region_ninp(g, true);
        if (!sst) continue;
        SML_REQUIRE(j < nslab && sids[j] == ids[i], "slab reservoir %d is not the rank's sst region %d (local %d)", j,
                    ids[i], i);
        int sninp = 0;
        if (int rc = sml_res_ninp(slab, j, &sninp)) return rc;
        SML_REQUIRE(sninp == 7 * in2d && soff[j + 1] - soff[j] == sninp,
                    "slab reservoir of region %d: %d inputs, the atmo subset has %d", ids[i], sninp, 7 * in2d);
        // atmo_training_data_idx (mod_slab_ocean_reservoir.f90:1550-1563): the lowest
        // level's 4 variables and logp, the sst, the tisr of the atmo feedback
        for (int e = natmo - kVars * in2d; e < natmo + in2d; ++e) ring_src.push_back((int32_t)(off[i] + e));
        for (int e = natmo + 2 * in2d; e < natmo + 4 * in2d; ++e) ring_src.push_back((int32_t)(off[i] + e));
        row.push_back(i);
        for (int p = 0; p < in2d; ++p) {  // the sst entries of the atmo feedback
            const int lx = p % g.inx, ly = p / g.inx;
            sfb.push_back((int32_t)(off[i] + natmo + 2 * in2d + p));
            sgrid.push_back(g2(input_x(g, lx + 1) - 1, g.in_ystart - 1 + ly));
            sreg.push_back((uint16_t)j);
        }
        ++j;
    }
    SML_REQUIRE(j == nslab, "%d slab reservoirs for %d sst regions", nslab, j);
    // wholegrid_sst point -> its region's exchange row and sst column
    const int xw = h->nout + snout;
    std::vector<int32_t> src(kGrid2d, -1);
    for (int r = 0; r < h->numregions; ++r) {
        RegionGeom g;
        region_geom(h->numregions, r, &g);
        for (int ly = 0; ly < g.resy; ++ly)
            for (int lx = 0; lx < g.resx; ++lx)
                src[g2(g.res_xstart - 1 + lx, g.res_ystart - 1 + ly)] = r * xw + h->nout + lx + g.resx * ly;
    }
    sml_hybrid::Slab &sl = h->slab;
    sl.nslab = nslab;
    sl.nsst = snout;
    sl.ratio = timestep_slab / timestep;
    sl.timestep = timestep;
    sl.timestep_slab = timestep_slab;
    sl.sst_bias = sst_bias;
    sl.base = d_base_sst;
    sl.mask = d_sea_mask;
    sl.tot_fb = (int)ring_src.size();
    sl.n_sst_el = (int)sfb.size();
    if (int rc = upload(&sl.d_ring_src, ring_src)) return rc;
    if (int rc = upload(&sl.d_row, row)) return rc;
    if (int rc = upload(&sl.d_sst_src, src)) return rc;
    if (int rc = upload(&sl.d_sfb, sfb)) return rc;
    if (int rc = upload(&sl.d_sgrid, sgrid)) return rc;
    if (int rc = upload(&sl.d_sreg, sreg)) return rc;
    if (hipMalloc(&sl.d_fb, std::max<size_t>(sl.tot_fb, 1) * 8) != hipSuccess ||
        hipMalloc(&sl.d_ov, std::max<size_t>((size_t)nslab * snout, 1) * 8) != hipSuccess ||
        hipMalloc(&sl.d_ring, std::max<size_t>((size_t)(sl.ratio - 1) * sl.tot_fb, 1) * 8) != hipSuccess ||
        hipMalloc(&sl.d_sst, (size_t)kGrid2d * 8) != hipSuccess ||
        hipMalloc(&sl.d_ms, std::max<size_t>((size_t)2 * nslab, 1) * 8) != hipSuccess)
        return fail(SML_ERR_NOMEM, "slab buffers");
    SML_HIP(hipMemset(sl.d_sst, 0, (size_t)kGrid2d * 8));
    h->xw = xw;
    if (int rc = sml_res_set_outvec_ld(h->res, xw)) return rc;
    if (h->res_cus > 0)  // the slab step runs on the main stream too
        if (int rc = sml_res_set_update_cus(slab, h->res_cus)) return rc;
    if (h->comm && (h->comm->world > 1 || h->force_exchange))
        if (int rc = alloc_exchange(h)) return rc;
    sl.res = slab;
    return SML_OK;
}

// start_prediction_slab's hand-over (mod_slab_ocean_reservoir.f90:769-800,
// parallelmain.f90:216-222): the slab reservoirs' sst [nslab][resx*resy] until their
// first prediction (the host synchronizes their states, sml_res_start_prediction);
// 272 K in the exchange rows of regions without a slab (mpires.f90:366-372); the
// ring of averaged inputs cleared (initialize_prediction_slab, :747-748).  After
// sml_hybrid_start, before the first step; the first step's exchange builds the SST.
extern "C" int sml_hybrid_start_slab(sml_hybrid *h, const double *d_slab_outvec) {
    SML_REQUIRE(h && h->slab.res, "sml_hybrid_set_slab first");
    SML_REQUIRE(h->ov && h->started, "sml_hybrid_start first");
    sml_hybrid::Slab &sl = h->slab;
    SML_REQUIRE(sl.nslab == 0 || d_slab_outvec, "null slab outvec");
    std::vector<double> ms(2 * std::max(sl.nslab, 1));
    for (int j = 0; j < sl.nslab; ++j) {
        double mean[36], stdv[36];
        if (int rc = sml_res_mean_std(sl.res, j, mean, stdv)) return rc;
        ms[2 * j] = mean[35];  // sst_mean_std_idx = the atmo grid's, 36 (mod_slab_ocean_reservoir.f90:1548)
        ms[2 * j + 1] = stdv[35];
    }
    hipStream_t m = h->main;
    if (sl.nslab)  // (a rank without sst regions has no slab mean / std)
        SML_HIP(hipMemcpyAsync(sl.d_ms, ms.data(), (size_t)2 * sl.nslab * 8, hipMemcpyHostToDevice, m));
    SML_HIP(hipMemsetAsync(sl.d_ring, 0, (size_t)(sl.ratio - 1) * sl.tot_fb * 8, m));
    const int nfill = h->nlocal * sl.nsst, n = sl.nslab * sl.nsst;
    hipLaunchKernelGGL(k_slab_rows, dim3((nfill + 255) / 256), dim3(256), 0, m, nullptr, nullptr, 0, sl.nsst, h->nlocal,
                       h->nout, h->xw, true, h->ov);
    if (n) {
        SML_HIP(hipMemcpyAsync(sl.d_ov, d_slab_outvec, (size_t)n * 8, hipMemcpyDeviceToDevice, m));
        hipLaunchKernelGGL(k_slab_rows, dim3((n + 255) / 256), dim3(256), 0, m, sl.d_ov, sl.d_row, sl.nslab, sl.nsst,
                           h->nlocal, h->nout, h->xw, false, h->ov);
    }
    SML_HIP(hipGetLastError());
    SML_HIP(hipStreamSynchronize(m));
    sl.dirty = true;
    sl.started = true;
    return SML_OK;
}

// the exchange row length: nout, or nout + the slab sst of the region's points
extern "C" int sml_hybrid_exchange_width(const sml_hybrid *h, int *width) {
    SML_REQUIRE(h && width, "null argument");
    *width = h->xw;
    return SML_OK;
}

// the slab state for hosts and tests: wholegrid_sst(96, 48) of the last exchange, the
// ring [timestep_slab/timestep - 1][tot] of averaged inputs (tot = *ring_len), the
// last slab feedback and slab outvecs [nslab][resx*resy]
extern "C" int sml_hybrid_slab_buffers(const sml_hybrid *h, const double **d_sst_grid, const double **d_ring,
                                       int *ring_len, const double **d_slab_feedback, const double **d_slab_outvec) {
    SML_REQUIRE(h && h->slab.res, "no slab ocean in this loop");
    const sml_hybrid::Slab &sl = h->slab;
    if (d_sst_grid) *d_sst_grid = sl.d_sst;
    if (d_ring) *d_ring = sl.d_ring;
    if (ring_len) *ring_len = sl.tot_fb;
    if (d_slab_feedback) *d_slab_feedback = sl.d_fb;
    if (d_slab_outvec) *d_slab_outvec = sl.d_ov;
    return SML_OK;
}

// predict for every local region (parallelmain.f90:225-234): the local outvecs in
// d_outvec on the main stream; with `assemble` (sml_hybrid_step on one rank) the
// finish also scatters them into the global grids
namespace {
int predict_impl(sml_hybrid *h, bool assemble) {
    SML_REQUIRE(h, "null context");
    if (!h->started) return fail(SML_ERR_STATE, "sml_hybrid_start first");
    if (h->predicted) return fail(SML_ERR_STATE, "sml_hybrid_predict twice without sml_hybrid_advance");
    h->assembled = false;
    if (h->overlap) {
        // (pipelined: the previous advance issued it already, unless the host discarded
        // it since -- sml_res_set_state / sml_res_step_cancel)
        int begun = 0;
        if (h->begun_next)
            if (int rc = sml_res_step_begun(h->res, &begun)) return rc;
        if (!begun)
            if (int rc = sml_res_step_begin(h->res, h->fb, h->main)) return rc;
        h->begun_next = false;
        if (int rc = slab_predict(h)) return rc;
        hipStream_t xs = h->main;
        if (h->chain) {  // the finish follows the window on SPEEDY's stream, once the begin is done
            xs = h->side;
            if (int rc = hop_signal(h, sml_hybrid::kHopBegun, h->main)) return rc;
            if (h->use_kernels && h->nlocal > 0) {  // waited for inside the finish (no wait kernel)
                if (int rc = sml::res_finish_wait(h->res, h->d_seq + sml_hybrid::kHopBegun * sml_hybrid::kSeqStride,
                                                  h->seq[sml_hybrid::kHopBegun], hop_late_word(h), h->hop_timeout))
                    return rc;
            } else if (int rc = hop_wait(h, sml_hybrid::kHopBegun, xs)) {
                return rc;
            }
        } else if (h->use_kernels && h->nlocal > 0) {
            // SPEEDY's forecast of the previous window, waited for inside the finish: its
            // weights load while the window runs (k_res_finish_grid's wflag; the main
            // stream's later work still follows the finish, so it follows the window too).
            // The finish's blocks spin on the reservoir's CUs, and the window's exit (the
            // forecast's producer) waits for its safety check, which runs on those CUs:
            // the finish launches only once that check is done (a CP wait on the main
            // stream, satisfied while the window still runs), or a host that enqueues
            // steps without polling run_speedy could starve the check behind the finish
            void *ev = nullptr;
            if (int rc = sml::dyn_check_event(h->dyn, &ev)) return rc;
            if (ev) SML_HIP(hipStreamWaitEvent(h->main, (hipEvent_t)ev, 0));
            if (int rc = sml::res_finish_wait(h->res, h->d_seq + sml_hybrid::kHopLm * sml_hybrid::kSeqStride,
                                              h->seq[sml_hybrid::kHopLm], hop_late_word(h), h->hop_timeout))
                return rc;
        } else if (int rc = hop_wait(h, sml_hybrid::kHopLm, h->main)) {  // SPEEDY's forecast of the previous window
            return rc;
        }
        // the local-model tiling fused into the v_p finish: one launch fewer on the
        // critical path; on one rank the assembly too (one more)
        if (assemble) {
            if (int rc = sml_res_step_finish_assemble(h->res, h->f4, h->f2, h->lm, h->ov, h->g4, h->g2, h->pr, xs))
                return rc;
            h->assembled = true;
        } else if (int rc = sml_res_step_finish_grid(h->res, h->f4, h->f2, h->lm, h->ov, xs)) {
            return rc;
        }
    } else {  // one pass over W_out: the same sums as begin + finish
        if (int rc = sml_res_step(h->res, h->fb, h->lm, h->ov, h->main)) return rc;
        if (int rc = slab_predict(h)) return rc;
    }
    h->predicted = true;
    return SML_OK;
}
}  // namespace

extern "C" int sml_hybrid_predict(sml_hybrid *h) { return predict_impl(h, false); }

// sendrecievegrid's assembly + run_model + re-tiling (mpires.f90:300-751) from the
// outvecs of every region in global region order ([numregions][nout], device)
extern "C" int sml_hybrid_advance(sml_hybrid *h, const double *d_outvec_all) {
    SML_REQUIRE(h && d_outvec_all, "null argument");
    if (!h->predicted) return fail(SML_ERR_STATE, "sml_hybrid_advance without sml_hybrid_predict");
    hipStream_t m = h->main, s = h->side;
    // the assembly's stream: the main stream (two hops around the window), or SPEEDY's,
    // right behind the window (sml_hybrid_set_chain); the re-tiling is the main stream's
    hipStream_t c = h->chain ? s : m;
    const bool hops = h->overlap && !h->chain;
    // (sml_hybrid_step on one rank: its predict assembled these very outvecs already)
    const bool done = h->assembled && d_outvec_all == h->ov;
    h->assembled = false;
    if (!done)
        if (int rc = sml_exchange_assemble(h->res, d_outvec_all, h->g4, h->g2, h->pr, c)) return rc;
    const bool sst_new = h->slab.res && h->slab.dirty;  // a new hybrid SST reaches sst_am this step
    if (int rc = slab_sst(h, d_outvec_all, c)) return rc;
    if (h->cal_on) {
        // run_model's date for this step (mpires.f90:1545, timestep = t + 1; before the
        // tisr lookup below, as the reference's calls meet the February latch) and the
        // window's forcing at that date (agcm_init, ini_agcm_init.f90:57-89), after the
        // previous window (the finish waited for its forecast) and any new hybrid SST
        int date[4];
        if (int rc = sml_calendar_delta_hour(h->tisr_startyear, h->tisr_base + (h->t + 1) * h->tisr_step_hours,
                                             &h->tisr_feb29, date))
            return rc;
        // on SPEEDY's stream, behind the previous window and beside the finish / assembly,
        // unless this step's new SST (written on c) must reach qcorh first
        if (int rc = sml_dyn_fordate(h->dyn, date[0], date[1], date[2], sst_new ? c : s)) return rc;
    }
    // chain on SPEEDY's stream with kernel hops: the next run_model's entry specx signals
    // the assembled grid as it starts (no signal kernel in front of the window); run_model
    // is then enqueued before the main stream's wait for that signal -- every in-kernel
    // wait is enqueued after its producer, so no wait can hold a hardware queue that its
    // producer sits behind
    const bool entry_sig = h->overlap && h->chain && h->use_kernels;
    if (entry_sig) {
        int adds = 0;
        if (int rc = sml::dyn_run_model_entry_signal(h->dyn, h->d_seq + sml_hybrid::kHopGrid * sml_hybrid::kSeqStride,
                                                     &adds))
            return rc;
        h->seq[sml_hybrid::kHopGrid] += (uint64_t)adds;
        if (int rc = sml_dyn_run_model(h->dyn, h->g4, h->g2, h->nleap, h->delt, h->alph, h->rob, h->wil, h->f4, h->f2,
                                       s))
            return rc;
    } else if (h->overlap) {  // the assembled grid: to SPEEDY's stream (two-stream) / to the main stream (chain)
        if (int rc = hop_signal(h, sml_hybrid::kHopGrid, c)) return rc;
    }
    if (h->chain)
        if (int rc = hop_wait(h, sml_hybrid::kHopGrid, m)) return rc;
    ++h->t;
    if (int rc = sml_res_tile_feedback(h->res, h->g4, h->g2, h->pr, h->tisr_table ? nullptr : h->tisr, h->fb, m))
        return rc;
    if (h->tisr_table) {  // get_tisr_by_date(..., timestep - 1, ...) for the next feedback (mpires.f90:726-728)
        int idx = 0;
        if (int rc = sml_tisr_date_index(h->tisr_startyear, h->tisr_base + (h->t - 1) * h->tisr_step_hours,
                                         &h->tisr_feb29, &idx))
            return rc;
        if (idx < 1 || idx > h->tisr_nhours)
            return fail(SML_ERR_ARG, "tisr hour %d outside the table's %d hours", idx, h->tisr_nhours);
        if (int rc = sml_res_tile_tisr_field(h->res, h->tisr_table + (size_t)(idx - 1) * kGrid2d, h->fb, m))
            return rc;
    }
    if (h->slab.res && h->slab.tot_fb) {  // averaged_atmo_input_vec(:, mod(t-1, R-1)+1), mpires.f90:755
        sml_hybrid::Slab &sl = h->slab;
        double *col = sl.d_ring + (size_t)((h->t - 1) % (sl.ratio - 1)) * sl.tot_fb;
        hipLaunchKernelGGL(k_slab_ring, dim3((sl.tot_fb + 255) / 256), dim3(256), 0, m, h->fb, sl.d_ring_src, sl.tot_fb,
                           col);
        SML_HIP(hipGetLastError());
    }
    if (hops) {
        if (h->use_kernels) {  // the entry's specx waits for the assembled grid in-kernel
            if (int rc = sml::dyn_run_model_wait(h->dyn, h->d_seq + sml_hybrid::kHopGrid * sml_hybrid::kSeqStride,
                                                 h->seq[sml_hybrid::kHopGrid], hop_late_word(h), h->hop_timeout))
                return rc;
        } else if (int rc = hop_wait(h, sml_hybrid::kHopGrid, s)) {
            return rc;
        }
    }
    // kernel hops: the forecast's signal is a store that run_model issues right behind
    // its exit (inside the window graph when the exit is captured there); the loop's
    // sequence number moves only once run_model is enqueued, so a run_model that fails
    // leaves no store pending and no finish waiting for one.  (The exit's own blocks
    // signalling instead, an agent-scope release each, measured no faster: DESIGN.md §4c)
    const bool exit_store = hops && h->use_kernels;
    const uint64_t lm_next = h->seq[sml_hybrid::kHopLm] + 1;
    if (exit_store)
        if (int rc = sml::dyn_run_model_exit_store(h->dyn, h->d_seq + sml_hybrid::kHopLm * sml_hybrid::kSeqStride,
                                                   lm_next))
            return rc;
    if (!entry_sig)
        if (int rc = sml_dyn_run_model(h->dyn, h->g4, h->g2, h->nleap, h->delt, h->alph, h->rob, h->wil, h->f4, h->f2,
                                       s)) {
            if (exit_store) (void)sml::dyn_run_model_exit_store(h->dyn, nullptr, 0);
            return rc;
        }
    if (exit_store) h->seq[sml_hybrid::kHopLm] = lm_next;
    if (hops && !exit_store) {
        if (int rc = hop_signal(h, sml_hybrid::kHopLm, s)) return rc;
    } else if (!h->overlap && h->ncs) {
        if (int rc = sml_res_tile_local_model(h->res, h->f4, h->f2, h->lm, s)) return rc;
    }
    // pipelined: the next step's begin from the feedback just tiled, on the main stream,
    // beside this window (it would be the next predict's first launch anyway)
    if (h->pipelined && h->overlap) {
        if (int rc = sml_res_step_begin(h->res, h->fb, m)) return rc;
        h->begun_next = true;
    }
    h->predicted = false;
    h->advanced = true;
    return SML_OK;
}

// advance from the all-gather's output d_recv[world][maxc][nout] (sml_exchange_plan):
// the slabs are global region order with even shares, else k_gather_rows permutes
// them into it first (on the main stream)
extern "C" int sml_hybrid_advance_slabs(sml_hybrid *h, const double *d_recv) {
    SML_REQUIRE(h && d_recv, "null argument");
    const int world = h->comm ? h->comm->world : 1;
    if (world == 1 || h->contiguous) return sml_hybrid_advance(h, d_recv);  // slabs in region order
    if (!h->predicted) return fail(SML_ERR_STATE, "sml_hybrid_advance_slabs without sml_hybrid_predict");
    const int total = h->numregions * h->xw;
    hipLaunchKernelGGL(k_gather_rows, dim3((total + 255) / 256), dim3(256), 0, h->chain ? h->side : h->main, d_recv,
                       h->d_perm, h->d_glob, h->xw, total);
    SML_HIP(hipGetLastError());
    return sml_hybrid_advance(h, h->d_glob);
}

// one hybrid step with the loop's own exchange: identity on one rank, else the
// all-gather of every rank's outvec slab (RCCL over xGMI) on the main stream
extern "C" int sml_hybrid_step(sml_hybrid *h) {
    SML_REQUIRE(h, "null context");
    if (int rc = hop_late_check(h, "sml_hybrid_step")) return rc;  // a host word: no sync
    const int world = h->comm ? h->comm->world : 1;
    if (world == 1 && h->nlocal != h->numregions)
        return fail(SML_ERR_STATE, "one rank holds %d of %d regions: exchange through sml_hybrid_advance",
                    h->nlocal, h->numregions);
    if (world > 1 && !h->comm->comm)
        return fail(SML_ERR_STATE, "rank %d of %d has no transport: exchange through sml_hybrid_advance_slabs",
                    h->comm->rank, world);
    // one rank: the exchange is the identity, so the finish assembles the grids itself;
    // forced, it goes through the transport as at world > 1
    const bool identity = world == 1 && !h->force_exchange;
    const bool fuse = identity && h->overlap && sml::res_in_global_order(h->res);
    if (int rc = predict_impl(h, fuse)) return rc;
    if (identity) return sml_hybrid_advance(h, h->ov);
    // (world > 1, or world 1 forced through the transport)
    // even shares (1152 / N for N = 1, 2, 4, 8): the outvecs go out of ov as they are;
    // uneven ones are padded to the largest share through d_send (one copy more on the
    // critical path; d_send's padding rows stay zero)
    hipStream_t xs = h->chain ? h->side : h->main;
    const double *send = h->ov;
    if (h->nlocal != h->maxc) {
        SML_HIP(hipMemcpyAsync(h->d_send, h->ov, (size_t)h->nlocal * h->xw * 8, hipMemcpyDeviceToDevice, xs));
        send = h->d_send;
    }
    if (int rc = sml_comm_allgather(h->comm, send, h->d_recv, (int64_t)h->maxc * h->xw, xs)) return rc;
    ++h->allgathers;
    return sml_hybrid_advance_slabs(h, h->d_recv);
}

extern "C" int sml_hybrid_exchanges(const sml_hybrid *h, int64_t *allgathers) {
    SML_REQUIRE(h && allgathers, "null argument");
    *allgathers = h->allgathers;
    return SML_OK;
}

// run_speedy after the last advance (mpires.f90:721, :1623): 0 ends the prediction
// (parallelmain.f90:268-270).  Waits for that step's safety check only.
extern "C" int sml_hybrid_run_speedy(sml_hybrid *h, int *run) {
    SML_REQUIRE(h && run, "null argument");
    if (!h->advanced) {
        *run = 1;
        return SML_OK;
    }
    if (int rc = sml_dyn_last_safe(h->dyn, run, nullptr)) return rc;
    // once that step's check is done, every wait of the step has run (the check follows
    // the entry specx -- behind k_io_entry, or behind the window's first row kernel's go
    // when the entry is inside the window graph -- which follows the finish), or the
    // check's own hand-off gave up (reported below): a wait that gave up fails the step
    // here, so a host polling per step (parallelmain.f90:268-270) stops instead of
    // going on from NaN forecasts; run_speedy is then 0
    if (int rc = hop_late_check(h, "sml_hybrid_run_speedy")) {
        *run = 0;
        return rc;
    }
    if (int rc = sml::dyn_check_late(h->dyn)) {
        *run = 0;
        return rc;
    }
    return SML_OK;
}

// wait for every issued step; the local model of the last window is tiled as the
// one-stream loop leaves it (the overlapped loop tiles it inside the next finish)
extern "C" int sml_hybrid_sync(sml_hybrid *h) {
    SML_REQUIRE(h, "null context");
    if (h->overlap && h->advanced && h->ncs) {
        if (h->chain) {
            if (int rc = sml_res_tile_local_model(h->res, h->f4, h->f2, h->lm, h->side)) return rc;
        } else {
            if (int rc = hop_wait(h, sml_hybrid::kHopLm, h->main)) return rc;
            if (int rc = sml_res_tile_local_model(h->res, h->f4, h->f2, h->lm, h->main)) return rc;
        }
    }
    SML_HIP(hipStreamSynchronize(h->main));
    SML_HIP(hipStreamSynchronize(h->side));
    if (int rc = hop_late_check(h, "sml_hybrid_sync")) return rc;
    return sml::dyn_check_late(h->dyn);
}

// ------------------------------------------------------------- diagnostics
// The step-accounting timeline (sml_timeline.hpp; profiling build only, -DSML_TL): a
// device buffer of per-(launch, block) start / end times of the step's kernels,
// attached to every translation unit; reset != 0 zeroes it (after the device is idle).
// *d_buf = the buffer (sml::tl::Buf), *bytes its size; SML_ERR_STATE in a build
// without the timeline.  Not in the public header (tools/probe_step_accounting.py).
extern "C" int sml_dbg_timeline(void **d_buf, int64_t *bytes, int reset) {
    SML_REQUIRE(d_buf && bytes, "null argument");
    static sml::tl::Buf *buf = nullptr;
    if (!buf) {
        sml::tl::Buf *b = nullptr;
        SML_HIP(hipMalloc(&b, sizeof(sml::tl::Buf)));
        if (sml::tl_attach_dynamics(b) || sml::tl_attach_spectral(b) || sml::tl_attach_reservoir(b) ||
            sml::tl_attach_hybrid(b)) {
            (void)hipFree(b);
            return fail(SML_ERR_STATE, "this build has no step timeline (compile with -DSML_TL)");
        }
        buf = b;
        reset = 1;
    }
    if (reset) {
        SML_HIP(hipDeviceSynchronize());
        SML_HIP(hipMemset(buf, 0, sizeof(sml::tl::Buf)));
        SML_HIP(hipDeviceSynchronize());
    }
    *d_buf = buf;
    *bytes = (int64_t)sizeof(sml::tl::Buf);
    return SML_OK;
}

// ------------------------------------------------------------- device memory
// plumbing for hosts without a GPU runtime binding of their own (the Fortran host):
// zeroed device allocations and synchronous copies
extern "C" int sml_device_alloc(int64_t bytes, void **d_ptr) {
    SML_REQUIRE(d_ptr && bytes >= 0, "bad argument");
    *d_ptr = nullptr;
    SML_HIP(hipMalloc(d_ptr, bytes > 0 ? (size_t)bytes : 16));
    SML_HIP(hipMemset(*d_ptr, 0, bytes > 0 ? (size_t)bytes : 16));
    return SML_OK;
}

extern "C" int sml_device_free(void *d_ptr) {
    if (d_ptr) SML_HIP(hipFree(d_ptr));
    return SML_OK;
}

extern "C" int sml_copy_to_device(void *d_dst, const void *src, int64_t bytes) {
    SML_REQUIRE(d_dst && src && bytes >= 0, "bad argument");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(d_dst, src, (size_t)bytes, hipMemcpyHostToDevice));
    return SML_OK;
}

extern "C" int sml_copy_to_host(void *dst, const void *d_src, int64_t bytes) {
    SML_REQUIRE(dst && d_src && bytes >= 0, "bad argument");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(dst, d_src, (size_t)bytes, hipMemcpyDeviceToHost));
    return SML_OK;
}

// region geometry of the res_domain decomposition (getxyresextent, getoverlapindices;
// res_domain.f90:123-204), 1-based like the reference:
// g[12] = res_xstart, res_xend, res_ystart, res_yend, resx, resy, in_xstart, in_xend,
//         in_ystart, in_yend, inx, iny
extern "C" int sml_region_geometry(int numregions, int region, int *g) {
    SML_REQUIRE(g, "null argument");
    RegionGeom r;
    SML_REQUIRE(region_geom(numregions, region, &r), "region %d of %d does not decompose the grid", region,
                numregions);
    const int v[12] = {r.res_xstart, r.res_xend, r.res_ystart, r.res_yend, r.resx, r.resy,
                       r.in_xstart,  r.in_xend,  r.in_ystart,  r.in_yend,  r.inx,  r.iny};
    std::memcpy(g, v, sizeof v);
    return SML_OK;
}

// processor_decomposition (res_domain.f90:31-62): the regions (0-based) rank irank of
// numprocs owns; returns their count in *count (regions may be NULL to ask only)
extern "C" int sml_processor_decomposition(int numregions, int numprocs, int irank, int *regions, int *count) {
    SML_REQUIRE(count && numregions > 0 && numprocs > 0 && irank >= 0 && irank < numprocs, "bad argument");
    std::vector<int> r(numregions);
    *count = processor_regions(numregions, numprocs, irank, r.data());
    if (regions) std::memcpy(regions, r.data(), sizeof(int) * *count);
    return SML_OK;
}
