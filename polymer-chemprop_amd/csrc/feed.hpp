// feed.hpp — native streamed batches (BASELINE.json configs[4]: millions of synthetic polymer graphs per
// rank, never materialised).  Host-side engine behind wdmpnn_feed_* (include/wdmpnn.h):
//
//   producer threads            feed thread (its own HIP stream)             consumer (caller's stream)
//   generate + plan + stage  -> H2D of the staged image + graph build  ->  wait on the graph's ready
//   into pinned slot i % R      into device slot i % R, ready event          event, encode, release
//
// Batch i is generated from seed + i (the caller mixes the rank into the seed: disjoint shards), goes
// through host slot i % R and device slot i % R, and is handed out in order.  A host slot is rewritten
// only after the H2D that read it has completed (its copy event, waited on by the producer); a device
// slot only after the consumer's work on its previous batch (the release event, waited on by the feeder
// thread with hipEventSynchronize: the feeder runs several batches ahead, so the host wait costs nothing,
// while a feed-stream wait on the consumer's event cost the consumer's stream ~60 us per training step).
// The caller's thread never blocks on either.  No Python, no GIL: the caller's thread only takes
// finished graphs.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "compact.hpp"
#include "graph_build.hpp"
#include "wdmpnn.h"

// (wdmpnn.hip) the build parameters / WdGraph of a compact batch, and one launch for several builds
int graph_build_prepare(const WdCompact *c, void *buffer, size_t bytes, int32_t flags, wd::GraphBuildP &P, WdGraph &Gout);
int graph_build_launch(const wd::GraphBuildP *P, int n, hipStream_t st);

namespace wd {

// upper bounds of one batch of `batch` generated graphs of `kind` (compact::generate)
struct FeedBounds { int atoms_per_mol, pairs_per_mol; };
inline FeedBounds feed_bounds(int kind) {
    // skeleton: n - 1 chain bonds + n / 5 ring closures; polymer: two monomers of <= 24 atoms + 10 rules
    if (kind == 0) return {48, 47 + 9 + 10};
    if (kind == 1) return {9, 8 + 1};
    return {37, 36 + 7};
}
inline size_t feed_host_bytes(int kind, int batch) {
    const FeedBounds f = feed_bounds(kind);
    const size_t V = (size_t)batch * f.atoms_per_mol + 1, P = (size_t)batch * f.pairs_per_mol;
    // mols [B][4] int32 + xn [B] + atoms + pairs + blocks [<= B][8] + block_nnz [<= B][2], 256-aligned each
    return 16 * (size_t)batch + 4 * (size_t)batch + sizeof(WdAtomCode) * V + sizeof(WdBondPair) * P +
           32 * (size_t)batch + 8 * (size_t)batch + 7 * 256;
}
constexpr int FEED_MAX_DEG = 24;  // bound of the mean in-degree used to size a slot's gather lists

struct Feed {
    WdFeedSpec spec{};
    hipStream_t fs = nullptr;
    int R = 0;
    size_t host_bytes = 0, dev_bytes = 0, graph_off = 0;
    struct Slot {
        int64_t turn = 0;       // producer: the batch allowed to write this host slot next
        int64_t staged = -1;    // batch staged in the host slot
        int counts[6] = {};     // n_mols, n_atoms, n_bonds, n_blocks, nnz_msg, nnz_agg
        size_t off[6] = {}, total = 0;
        bool copy_pending = false;
        int64_t built = -1;     // batch whose device graph is enqueued (ready event recorded)
        WdGraph g{};
        hipEvent_t copy_done = nullptr, ready = nullptr, released = nullptr;
    };
    std::vector<Slot> slot;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::thread> threads;
    int64_t handed = 0;         // consumer: batches handed out
    int64_t released_upto = 0;  // batches [0, released_upto) released (their release events recorded)
    bool stop = false;
    std::string error;

    uint8_t *host(int s) const { return (uint8_t *)spec.pinned + (size_t)s * host_bytes; }
    uint8_t *dev(int s) const { return (uint8_t *)spec.device + (size_t)s * dev_bytes; }

    void fail_locked(const std::string &e) {
        if (error.empty()) error = e;
        stop = true;
        cv.notify_all();
    }

    void producer(int t) {
        try {
            compact::Batch c;  // reused: no allocation per batch once the vectors have grown
            compact::Plan p;
            for (int64_t i = t; i < spec.n_batches; i += spec.producers) {
                const int s = (int)(i % R);
                Slot &S = slot[(size_t)s];
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || S.turn == i; });
                    if (stop) return;
                }
                if (S.copy_pending && hipEventSynchronize(S.copy_done) != hipSuccess) throw std::runtime_error("copy event");
                compact::generate(spec.kind, spec.batch, spec.seed + (uint64_t)i, c);
                c.fa = spec.atom_fdim;
                c.fb = spec.bond_fdim;
                if (!compact::plan(c, spec.target_blocks, p)) throw std::runtime_error("generated molecule exceeds a block");
                const compact::Staged st = compact::stage_layout(c, p);
                if (st.total > host_bytes) throw std::runtime_error("staged batch larger than its slot");
                compact::stage_copy(c, p, st, host(s));
                std::lock_guard<std::mutex> lk(mu);
                const int cnt[6] = {c.n_mols(), c.n_atoms(), c.n_bonds(), p.n_blocks(), (int)p.nnz_msg, (int)p.nnz_agg};
                std::copy(cnt, cnt + 6, S.counts);
                std::copy(st.off, st.off + 6, S.off);
                S.total = st.total;
                S.staged = i;
                cv.notify_all();
            }
        } catch (const std::exception &e) {
            std::lock_guard<std::mutex> lk(mu);
            fail_locked(std::string("feed producer: ") + e.what());
        }
    }

    // batch i is ready for the feed thread: staged, and its device slot's previous batch released
    bool feedable(int64_t i) const {
        const Slot &S = slot[(size_t)(i % R)];
        return S.staged == i && released_upto >= i - R + 1;
    }

    // Batches go through in groups: every batch already staged (up to WD_MULTI) is uploaded, and their
    // graphs are built by ONE launch (graph_build_launch): a build is a short launch of one workgroup per
    // molecule block, so several batches per launch keep more CUs busy for the same latency.
    void feeder() {
        try {
            std::vector<GraphBuildP> P;
            std::vector<WdGraph> G;
#ifndef WD_FEED_GROUP
#define WD_FEED_GROUP 1
#endif
            // a group of grp batches per build launch while the consumer has two or more built batches in
            // hand (waking for every staged batch gave launches of one batch): streamed leg 146.2-155.9
            // against 142.0-149.3 M edges/s, same box, three rounds (WD_FEED_GROUP=0: the old wake-up)
            const int64_t grp = WD_FEED_GROUP ? std::min<int64_t>(WD_MULTI, std::max<int64_t>(1, R / 2)) : 1;
            for (int64_t i = 0; i < spec.n_batches;) {
                int64_t n = 0;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] {
                        return stop || (feedable(i) && (grp == 1 || i + grp > spec.n_batches || feedable(i + grp - 1) ||
                                                        i - handed < 2));
                    });
                    if (stop) return;
                    while (n < WD_MULTI && i + n < spec.n_batches && feedable(i + n)) ++n;
                }
                P.assign((size_t)n, GraphBuildP{});
                G.assign((size_t)n, WdGraph{});
                for (int64_t j = 0; j < n; ++j) {
                    const int s = (int)((i + j) % R);
                    Slot &S = slot[(size_t)s];
                    // the slot's previous batch released: waited for on this (feeder) thread, not with a
                    // stream wait of the feed stream on the consumer's event -- that cross-stream dependency
                    // cost the consumer's stream ~60 us per training step (streamed training 0.46 ms
                    // against 0.40 resident; 0.41 with the host wait, same box, tools/train_stream_host.py)
                    if (i + j >= R && hipEventSynchronize(S.released) != hipSuccess)
                        throw std::runtime_error("release wait");
                    if (hipMemcpyAsync(dev(s), host(s), S.total, hipMemcpyHostToDevice, fs) != hipSuccess ||
                        hipEventRecord(S.copy_done, fs) != hipSuccess)
                        throw std::runtime_error("H2D");
                    WdCompact c{};
                    c.n_mols = S.counts[0]; c.n_atoms = S.counts[1]; c.n_bonds = S.counts[2]; c.n_blocks = S.counts[3];
                    c.atom_fdim = spec.atom_fdim; c.bond_fdim = spec.bond_fdim;
                    c.nnz_msg = S.counts[4]; c.nnz_agg = S.counts[5];
                    uint8_t *d = dev(s);
                    c.mols = (const int32_t *)(d + S.off[0]); c.xn = (const float *)(d + S.off[1]);
                    c.atoms = (const WdAtomCode *)(d + S.off[2]); c.pairs = (const WdBondPair *)(d + S.off[3]);
                    c.blocks = (const int32_t *)(d + S.off[4]); c.block_nnz = (const int32_t *)(d + S.off[5]);
                    if (graph_build_prepare(&c, d + graph_off, dev_bytes - graph_off, spec.flags, P[(size_t)j], G[(size_t)j]))
                        throw std::runtime_error(std::string("graph build: ") + wdmpnn_last_error());
                }
                if (graph_build_launch(P.data(), (int)n, fs))
                    throw std::runtime_error(std::string("graph build: ") + wdmpnn_last_error());
                for (int64_t j = 0; j < n; ++j)
                    if (hipEventRecord(slot[(size_t)((i + j) % R)].ready, fs) != hipSuccess) throw std::runtime_error("ready event");
                std::lock_guard<std::mutex> lk(mu);
                for (int64_t j = 0; j < n; ++j) {
                    Slot &S = slot[(size_t)((i + j) % R)];
                    S.copy_pending = true;
                    S.turn = i + j + R;  // the producer of batch i + j + R waits for copy_done itself
                    S.g = G[(size_t)j];
                    S.built = i + j;
                }
                cv.notify_all();
                i += n;
            }
        } catch (const std::exception &e) {
            std::lock_guard<std::mutex> lk(mu);
            fail_locked(std::string("feed: ") + e.what());
        }
    }

    void shutdown() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        for (auto &t : threads)
            if (t.joinable()) t.join();
        threads.clear();
        if (fs) (void)hipStreamSynchronize(fs);
    }

    ~Feed() {
        shutdown();
        for (auto &S : slot) {
            if (S.copy_done) (void)hipEventDestroy(S.copy_done);
            if (S.ready) (void)hipEventDestroy(S.ready);
            if (S.released) (void)hipEventDestroy(S.released);
        }
        if (fs) (void)hipStreamDestroy(fs);
    }
};

}  // namespace wd
