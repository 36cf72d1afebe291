/*
 * aidfp.h -- C ABI of the MI355X fingerprint engine (libaidfp.so, gfx950).
 *
 * This is the drop-in boundary that replaces the process boundary of the
 * reference: audio-ident-service/app/audio/fingerprint.py spawns `olaf_c`
 * (store :117-125, query :185-193, del :239-246) with env OLAF_DB (:71-84) and
 * parses its stdout CSV (:273-350). Here the same three operations are plain C
 * calls on caller-owned buffers; the Python adapter
 * (audio-ident_amd/aidfp/fingerprint.py) keeps the reference's async API on top.
 *
 * Conventions: every function returns AID_OK (0) or a negative AID_ERR_*;
 * aid_last_error() returns a thread-local message for the last failure. Pointers
 * are plain host or device pointers as documented per call; `stream` is a
 * hipStream_t passed as void* (NULL = the engine's own stream, a blocking stream:
 * it is ordered after work the caller queued on the legacy default stream, so
 * buffers produced there are complete before the engine reads them). An engine is
 * bound to one GPU and takes an internal lock per call, so calls from several
 * threads never corrupt it; but a SEQUENCE of calls that shares state (aid_extract
 * then aid_result_* / aid_index_add_extracted / aid_query_extracted) must not be
 * interleaved with another thread's extraction. The single-call readers aid_query_pcm
 * and aid_exact_lane have no such window. The Python adapter takes a reader/writer
 * lock: index writers exclusive (the reference's single LMDB writer,
 * fingerprint.py:7-8), concurrent readers shared.
 */
#ifndef AIDFP_H
#define AIDFP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AID_ABI_VERSION 1

#define AID_OK 0
#define AID_ERR_INVALID (-1)  /* bad argument */
#define AID_ERR_DEVICE (-2)   /* HIP runtime / device failure: engine unusable */
#define AID_ERR_NOMEM (-3)    /* device or host allocation failed */
#define AID_ERR_STATE (-4)    /* call out of order (e.g. no extraction yet) */

#define AID_PCM_HOST 0
#define AID_PCM_DEVICE 1

/* kernel ids for aid_profile_read */
#define AID_K_STFT 0
#define AID_K_PEAKS 1
#define AID_K_LANDMARK_COUNT 2
#define AID_K_LANDMARK_WRITE 3
#define AID_K_SYNTH 4
#define AID_K_MATCH 5
#define AID_K_RESAMPLE 6
#define AID_K_DEDUP 7
#define AID_K_INDEX_BUILD 8 /* the K4 sort build (sort + bucket lengths + offsets) */
#define AID_K_VOTE_HIST 9    /* K5a: seen filter + global vote histogram (global match path) */
#define AID_K_HOT_SCAN 10    /* K5h: histogram rows -> hot-bucket bitmaps */
#define AID_K_VOTE_FINAL 11  /* K5b: exact (track, d) table of the hot votes, best d per track, rows */
#define AID_K_COUNT 12       /* AID_K_MATCH (5) is the LDS match path (k_match_lds) */

typedef struct aid_engine aid_engine;

typedef struct aid_config {
    int32_t sample_rate;   /* Hz; per-index property */
    int32_t hop;           /* 0 = FPSPEC default: 512 at sr >= 32 kHz, else 256 */
    float peak_threshold;  /* 0 = FPSPEC default 4.0; otherwise in [2^-124, 2^100] */
    int32_t device;        /* HIP device ordinal; -1 = current device */
    int32_t min_match;     /* query: 0 = FPSPEC default 10 (distinct query anchor frames, FPSPEC v1 7) */
    int32_t max_results;   /* query: 0 = FPSPEC default 50 */
    int32_t flags;         /* AID_FLAG_* (0 = default) */
    int32_t reserved[9];
} aid_config;

/* aid_config.flags: keep the whole power plane of an extraction for aid_result_power. Without it
   K1 skips the stores of 64-bin blocks whose every power is <= peak_threshold (K2 never reads
   them) and aid_result_power fails with AID_ERR_STATE. */
#define AID_FLAG_KEEP_POWER 1

/* one landmark record (FPSPEC 6): hash in the low word, anchor frame in the high word */
typedef struct aid_hash {
    uint32_t hash;
    uint32_t t1;
} aid_hash;

int32_t aid_abi_version(void);
const char *aid_last_error(void);

/* Fill *out with the FPSPEC defaults for `sample_rate`. */
int aid_config_default(int32_t sample_rate, aid_config *out);

/* Create / destroy an engine (allocates device tables; workspaces grow on demand). */
int aid_engine_create(const aid_config *cfg, aid_engine **out);
void aid_engine_destroy(aid_engine *e);
int aid_engine_config(const aid_engine *e, aid_config *out);

/* Test hook: force one of the engine's own code paths, which it otherwise chooses itself per call
   (the parity tests run every path against the oracle). Never needed in production. */
#define AID_FORCE_K5_PATH 1        /* 0 auto, 1 LDS vote table first, 2 global histogram only */
#define AID_FORCE_K5_PARTS 2       /* 0 by vote count, else 1, 2 or 4 key partitions per query (K5a) */
#define AID_FORCE_K5_BATCH 3       /* 0 default (2048), else global-path queries per launch */
#define AID_FORCE_K2_STRIPS_X100 4 /* 0 adaptive, else 100 x K2 strips per resident workgroup slot */
#define AID_FORCE_K4_BUILD 5       /* 0 default, 1 radix sort (the default), 2 atomic counting sort, 3 rocPRIM sort (A/B; only in the
                                      diagnostic variant library, else AID_ERR_INVALID),
                                      4 radix sort with the ballot-matched in-wave rank (A/B of the one-atomic rank) */
#define AID_FORCE_EXCHANGE_FAIL 6  /* 1: the next index exchange's pack (aid_index_pack, or the prepare step of
                                      aid_index_allgather) fails with AID_ERR_NOMEM, once (rank-failure tests) */
#define AID_FORCE_LANE_GATHER 7    /* 1: aid_exact_lane copies its sub-windows to a staging buffer before K1 instead
                                      of extracting them in place (A/B) */
#define AID_FORCE_PLANE_ROWS 8     /* 0 default (786,432), else power rows per K1 -> K2 clip group of one extraction
                                      call (tests: small calls split into several groups) */
int aid_engine_force(aid_engine *e, int32_t what, int32_t value);

/* Frames and worst-case record count of a clip of n samples (FPSPEC 1, 5). */
int64_t aid_num_frames(const aid_engine *e, int64_t n_samples);
int64_t aid_hash_capacity(const aid_engine *e, int64_t n_samples);

/*
 * Fingerprint extraction (K1 stft_power -> K2 peak_pick -> K3 landmark_hash).
 * Clip c is pcm[offsets[c] .. offsets[c+1]); `offsets` is a HOST array of
 * n_clips+1 non-decreasing sample indices. With AID_PCM_DEVICE, `pcm` is a device
 * pointer read in place (a clip at an odd offset reads its frames with 4-byte aligned
 * float2 loads); with AID_PCM_HOST the engine stages the samples itself, by ONE
 * asynchronous copy on `stream`: from page-locked memory that copy is a DMA, so
 * host PCM must stay unchanged until the call's stream completes (aid_sync, or
 * any aid_result_* call). An error return has already drained the stream.
 * Asynchronous on `stream`; results stay on the device until fetched below.
 * Replaces the FFT/peak/hash work of `olaf_c store|query` (fingerprint.py:117,185).
 */
int aid_extract(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t pcm_location,
                void *stream);

/* Block until the last extraction finished. */
int aid_sync(aid_engine *e);

/* Per-clip record counts of the last extraction (host array of n_clips). Synchronises. */
int aid_result_counts(aid_engine *e, int64_t *counts);
/* Copy clip `clip`'s records to host `out` (capacity `cap`); *n_out = count. Synchronises. */
int aid_result_hashes(aid_engine *e, int32_t clip, aid_hash *out, int64_t cap, int64_t *n_out);
/* Zero-copy device view of the last extraction: records (clip c starts at clip_base[c]),
   per-clip counts (device int64[n_clips]); clip_base is a HOST array owned by the engine. */
int aid_result_device(aid_engine *e, const aid_hash **records, const int64_t **counts_dev,
                      const int64_t **clip_base_host, int32_t *n_clips);

/* Debug/parity views of the last extraction (host copies, synchronise):
   power rows [F][1024] fp32 of clip `clip` (needs AID_FLAG_KEEP_POWER); peak bitmask [F][16] uint64. */
int aid_result_power(aid_engine *e, int32_t clip, float *out, int64_t cap_floats);
int aid_result_peakmask(aid_engine *e, int32_t clip, uint64_t *out, int64_t cap_words);

/* Log-magnitude spectrogram 10*log10(P + 1e-10) of one host clip: out[F][1024] (host). */
int aid_spectrogram(aid_engine *e, const float *pcm, int64_t n, float *out, int64_t cap_floats);

/* Deterministic synthetic PCM (aidfp/synth.py semantics) written to DEVICE `dst`
   [n_clips][n]: tracks/starts are HOST arrays; noise_a = query-noise half-width (0 = none). */
int aid_synth(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips, int64_t n,
              int32_t noise_a, uint32_t salt, void *stream);
/* Same with the partials' band [100, fmax_hz) Hz instead of [100, 8000) (fmax_hz <= sample_rate / 2): the
   bench's full-band workload, whose spectrum has no cold upper blocks. aid_synth = fmax_hz 8000. */
int aid_synth_band(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips,
                   int64_t n, int32_t noise_a, uint32_t salt, int32_t fmax_hz, void *stream);
/* Same audio at an explicit sample rate (the engine's own rate above): the same partials and notes sampled
   at `sample_rate`, e.g. a 44.1 kHz catalog or a 48 kHz capture for an engine that indexes at 16 kHz.
   flags: AID_SYNTH_STATIONARY = the v0 generator (constant amplitude within a note); default = v2 (every
   note decays linearly to half amplitude, as a struck or plucked note: landmark times lock to the onsets). */
#define AID_SYNTH_STATIONARY 1
/* flags: AID_SYNTH_ASYNC = return once the generation is enqueued on `stream` (ordered after the engine's
   earlier work on that stream; the caller orders its own reads of dst). Default: the call waits for it. */
#define AID_SYNTH_ASYNC 2
int aid_synth_rate(aid_engine *e, float *dst, const uint32_t *tracks, const int64_t *starts, int32_t n_clips,
                   int64_t n, int32_t sample_rate, int32_t noise_a, uint32_t salt, int32_t fmax_hz, int32_t flags,
                   void *stream);

/* ---- index + match (FPSPEC 7) ----
 * Replaces `olaf_c store` + LMDB (fingerprint.py:117-125), `olaf_c del` (:239-246) and
 * `olaf_c query` (:185-202). Postings accumulate on the device; the CSR is (re)built by
 * aid_index_finalize, which aid_query* call implicitly when the index changed. Single
 * writer: calls that mutate the index must be serialised by the caller (fingerprint.py:7-8). */

/* one query result row (FPSPEC 7): d = t_ref - t_q of the best offset bin, in frames */
typedef struct aid_match_row {
    int32_t match_count;
    uint32_t track;
    int32_t d;
    int32_t tq_min;
    int32_t tq_max;
} aid_match_row;

int aid_index_reset(aid_engine *e);
/* Add every clip of the last aid_extract as track track_ids[c] (host array of n_clips). Asynchronous: the
   clips' posting counts are scanned on the device and the call does not wait for them (only for the previous
   call's); every reader of the postings (stats, finalize, export, ...) waits for the count first. */
int aid_index_add_extracted(aid_engine *e, const uint32_t *track_ids);
/* Add n postings (hash, track, t) from host (AID_PCM_HOST) or device (AID_PCM_DEVICE) arrays. */
int aid_index_add_postings(aid_engine *e, const uint32_t *hash, const uint32_t *track, const uint32_t *t, int64_t n,
                           int32_t location);
/* Register track id `track` without postings (a clip too short or too quiet to give a hash), so a
 * later aid_index_remove of it succeeds like `olaf_c del` of any stored name (fingerprint.py:239-262).
 * Idempotent. */
int aid_index_add_track(aid_engine *e, uint32_t track);
/* Tombstone a track: its postings stop voting; AID_ERR_INVALID if unknown or already removed. */
int aid_index_remove(aid_engine *e, uint32_t track);
/* Drop the stored postings of every removed track (order of the others kept; the LMDB delete of
 * `olaf_c del` frees its entries). *n_removed = postings dropped. The CSR is rebuilt lazily. */
int aid_index_compact(aid_engine *e, int64_t *n_removed);
int aid_index_finalize(aid_engine *e);
/* Cumulative match counters since the last reset (the first n of 7): out[0] queries, [1] exact votes (postings whose
   hash a query record hits), [2] 8-B postings K5's global path read (once per key partition in K5a + once in K5b),
   [3] queries answered on the LDS path, [4] on the global path, [5] query records, [6] 2-B posting signatures the
   LDS path read (twice per vote: its counting and insert passes; the insert pass also reads the 8-B posting of a
   vote whose bucket is hot), [7] resident LDS-path workgroups per CU (an occupancy query, not a counter),
   [8..12] queries the LDS path handed to the global path, by reason: above 2^18 votes, (track, d) table full,
   distinct-frame set full, track table full, more rows than its staging holds. */
int aid_match_stats(aid_engine *e, int64_t *out, int32_t n, int32_t reset);
/* n_postings = stored postings, n_live = postings in the built CSR (-1 if stale), n_tracks = max id + 1 */
int aid_index_stats(aid_engine *e, int64_t *n_postings, int64_t *n_live, uint32_t *n_tracks);
/* Copy stored postings [first, first+count) to host or device columns (RCCL all-gather export). */
int aid_index_export(aid_engine *e, uint32_t *hash, uint32_t *track, uint32_t *t, int64_t first, int64_t count,
                     int32_t location);
/* Order-sensitive 64-bit checksum of stored postings [first, first+count), computed on the device:
   sum mod 2^64 over i of splitmix64-finalizer((hash << 32 | t) ^ track * 0x9E3779B97F4A7C15 ^ i * 0xD6E8FEB86659FD93),
   i counted from `first`. After the catalog exchange every rank compares its replica's checksum with the others'
   (the sequential ingest it replaces, app/ingest/pipeline.py:294-310, had one LMDB and nothing to compare). */
int aid_index_checksum(aid_engine *e, int64_t first, int64_t count, uint64_t *out);
/* The built CSR to host memory (tests and tools; the index must be finalized): offsets (n_offsets >= 2^26 + 1, or
   NULL) = the start of each bucket key's postings (offsets[k]..offsets[k+1]), posts (up to cap, or NULL) = the
   postings (track | t << 32) in bucket-key order, each bucket in arrival order (K4 is a stable sort); *n_out = the
   postings in the CSR (removed tracks' postings dropped). Replaces reading the LMDB that `olaf_c store` writes
   (audio-ident-service/app/audio/fingerprint.py:117-125). */
int aid_index_csr_export(aid_engine *e, uint32_t *offsets, int64_t n_offsets, uint64_t *posts, int64_t cap,
                         int64_t *n_out);
/* ---- PCM front-end (spec/FPSPEC.md 8) ----
 * Replaces ffmpeg `-ac 1 -ar <rate>` (audio-ident-service/app/audio/decode.py:41-60): optional
 * stereo downmix ((L+R)*0.5f) + rational polyphase resampling sr_in -> sr_out (scipy
 * resample_poly's Kaiser(5) filter, binary32, pinned order). src/dst are device pointers; src
 * holds n frames of `channels` (1, or 2 interleaved) floats, dst receives
 * aid_resample_len(n, sr_in, sr_out) mono samples. Asynchronous on `stream` (NULL = engine). */
int64_t aid_resample_len(int64_t n, int32_t sr_in, int32_t sr_out);
int aid_resample(aid_engine *e, const float *src, int64_t n, int32_t channels, int32_t sr_in, int32_t sr_out,
                 float *dst, int64_t cap, int64_t *n_out, void *stream);
/* Streaming form: src[0] is stream sample in_base (samples outside [in_base, in_base+n) read as 0);
 * computes stream outputs [m_first, m_first+count) into dst[0..count). Output m needs inputs up to
 * floor((m*down + hl)/up) and J-1 before it, so a caller that keeps that history gets exactly the
 * whole-signal result chunk by chunk (aidfp.stream). */
int aid_resample_range(aid_engine *e, const float *src, int64_t in_base, int64_t n, int32_t channels, int32_t sr_in,
                       int32_t sr_out, int64_t m_first, int64_t count, float *dst, void *stream);
/* aid_resample_range for n_streams streams in lockstep, ONE launch (config 5: every stream of a bank pushes
 * the same chunk length): stream i's input starts src_stride floats after stream i-1's, its outputs
 * dst_stride floats after. Each stream's outputs are bit for bit those of its own aid_resample_range.
 * Replaces one ffmpeg `-ac 1 -ar` process per upload (decode.py:41-60) for a whole batch of live streams. */
int aid_resample_batch(aid_engine *e, const float *src, int64_t src_stride, int32_t n_streams, int64_t in_base, int64_t n,
                       int32_t channels, int32_t sr_in, int32_t sr_out, int64_t m_first, int64_t count, float *dst,
                       int64_t dst_stride, void *stream);
/* aid_resample_batch over a two-part input: stream frames [in_base - hist_n, in_base) from hist (hist_stride floats
 * per stream), then [in_base, in_base + n) from src. A live stream's chunk is read where the caller holds it and only
 * the previous chunk's last few frames are kept, instead of appending every chunk to a long history first (a
 * 256-stream 2.5 s push is 246 MB of stereo: its append cost ~80 us of GPU per push). Outputs bit for bit those of
 * aid_resample_batch over the concatenated input. */
int aid_resample_batch_split(aid_engine *e, const float *hist, int64_t hist_stride, int64_t hist_n, const float *src,
                             int64_t src_stride, int32_t n_streams, int64_t in_base, int64_t n, int32_t channels,
                             int32_t sr_in, int32_t sr_out, int64_t m_first, int64_t count, float *dst,
                             int64_t dst_stride, void *stream);
/* (up, down, hl, J) of a rate pair (FPSPEC 8); returns 0 on bad rates */
int aid_resample_plan(int32_t sr_in, int32_t sr_out, int32_t *up, int32_t *down, int32_t *hl, int32_t *J);

/* ---- Chromaprint content dedup ----
 * Replaces app/audio/dedup.py:127-222 (`_fingerprint_similarity`, `check_content_duplicate`):
 * a device-resident catalog of raw Chromaprint fingerprints (u32 words) with durations; a scan
 * scores every entry whose duration d satisfies lo <= d <= hi (lo = duration*0.9,
 * hi = duration*1.1 in binary64, as the reference's SQL bounds) by
 * (matching_bits / (min_len*32)) * (min_len / max_len) in binary64 and returns the best entry
 * (earliest on ties, only scores > 0; -1 if none) and its score. Entry index = insertion order.
 * All arrays are host arrays; offsets are int64[n+1] word offsets. */
int aid_dedup_reset(aid_engine *e);
int aid_dedup_add(aid_engine *e, const uint32_t *words, const int64_t *offsets, const double *durations, int32_t n);
int aid_dedup_count(aid_engine *e, int64_t *n_entries, int64_t *n_words);
int aid_dedup_scan(aid_engine *e, const uint32_t *words, const int64_t *offsets, const double *durations, int32_t nq,
                   int64_t *best_idx, double *best_sim);
/* score of n (a_i, b_i) pairs, same formula (the reference's `_fingerprint_similarity`) */
int aid_dedup_pairs(aid_engine *e, const uint32_t *a, const int64_t *a_off, const uint32_t *b, const int64_t *b_off,
                    int32_t n, double *sim);

/* ---- native multi-GPU exchange (SURVEY.md 8b "aid_allgather_index", 8e) ----
 * One process per GPU. Rank 0 calls aid_comm_id, the host hands the 128 id bytes to every
 * rank (any side channel: torch.distributed store, MPI, a file), then every rank calls
 * aid_comm_create with its own engine. aid_comm wraps an RCCL communicator over xGMI.
 * Replaces the reference's single LMDB writer (pipeline.py:294-310, fingerprint.py:7-8):
 * ingest is sharded, the index is replicated by ONE all-gather. */
#define AID_COMM_ID_BYTES 128
typedef struct aid_comm aid_comm;
int aid_comm_id(uint8_t id[AID_COMM_ID_BYTES]);
int aid_comm_create(aid_engine *e, const uint8_t id[AID_COMM_ID_BYTES], int32_t world, int32_t rank, aid_comm **out);
void aid_comm_destroy(aid_comm *c);
/* Collective over all ranks of c: every rank's postings [first, n) (its shard) are all-gathered
 * (counts and track-id ranges first, then one padded SoA all-gather) and replace [first, n) by
 * the union in rank order; postings before `first` stay. The index is left dirty (finalize
 * next). *n_total = postings now held. Every rank must call it with the same comm.
 * Failure agreement: after the counts, every rank reserves the exchange buffers and the grown
 * index and packs its shard, then all ranks all-gather one ok flag; the payload all-gather runs
 * only if every rank is ready. A rank-local failure therefore makes EVERY rank return an error
 * (AID_ERR_STATE on the others) with its index unchanged, instead of leaving peers blocked in RCCL. */
int aid_index_allgather(aid_engine *e, aid_comm *c, int64_t first, int64_t *n_total);
/* The communicator's RCCL view: ranks (ncclCommCount) and this rank (ncclCommUserRank). */
int aid_comm_size(const aid_comm *c, int32_t *world, int32_t *rank);
/* aid_index_allgather in three steps, for an exchange the host runs itself (e.g. torch.distributed,
 * gloo on host copies). Every rank: aid_index_shard_info -> all-gather (count, n_tracks) -> stride = max
 * count -> aid_index_pack its shard into DEVICE planes [3][stride] (hash, track, t; zero padding) ->
 * all-gather the planes into DEVICE recv [world][3][stride] -> aid_index_splice with the host counts
 * [world] and max n_tracks. Splice is failure-atomic: on error the index is unchanged. */
int aid_index_shard_info(aid_engine *e, int64_t first, int64_t *count, uint32_t *n_tracks);
/* Everything a splice of `total` postings at `first` with n_tracks ids can fail on (growth of the posting
 * planes and the track tables), done ahead of the payload collective; the index itself does not change.
 * A host-driven exchange calls it with aid_index_pack before it agrees on every rank's readiness. */
int aid_index_reserve(aid_engine *e, int64_t first, int64_t total, uint32_t n_tracks, void *stream);
int aid_index_pack(aid_engine *e, int64_t first, uint32_t *planes, int64_t stride, void *stream);
int aid_index_splice(aid_engine *e, int64_t first, const uint32_t *recv, int32_t world, int64_t stride,
                     const int64_t *counts, uint32_t n_tracks, void *stream);

/* Flat versioned file (magic AIDFPIX1 + header + posting columns + tombstones): replaces the OLAF_DB dir. */
int aid_index_save(aid_engine *e, const char *path);
int aid_index_load(aid_engine *e, const char *path);
/* nq queries from host records: query q = recs[qoff[q] .. qoff[q+1]) (host qoff, nq+1 entries).
   rows: host [nq][max_results]; nrows: host [nq]. */
int aid_query(aid_engine *e, const aid_hash *recs, const int64_t *qoff, int32_t nq, aid_match_row *rows,
              int32_t *nrows);
/* Query with every clip of the last aid_extract (records stay on the device). */
int aid_query_extracted(aid_engine *e, aid_match_row *rows, int32_t *nrows);
/* Extraction + query of a batch of clips as ONE call (offsets/pcm as aid_extract; rows [n_clips][max_results],
   nrows [n_clips], host): safe to call from several threads at once -- the engine serialises the calls and no
   other call's extraction can interleave. The reader entry point of the Python service, which coalesces
   concurrent olaf_query requests into one call (replaces one `olaf_c query` process per request,
   fingerprint.py:185-193). Synchronous. */
int aid_query_pcm(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t pcm_location,
                  aid_match_row *rows, int32_t *nrows, void *stream);
/* aid_query_pcm over windows of DEVICE PCM given as [starts[c], ends[c]) sample ranges, which may overlap
 * (50 %-overlap stream windows, sub-windows of one clip): K1-K3 read them in place, then K5, in one critical
 * section. Rows as aid_query. Replaces one `olaf_c query` per window (fingerprint.py:185-193). */
int aid_query_windows(aid_engine *e, const float *pcm, const int64_t *starts, const int64_t *ends, int32_t n_windows,
                      aid_match_row *rows, int32_t *nrows, void *stream);
/* The same query in two halves (a caller overlaps its next batch's host work with this batch's
 * kernels). _submit enqueues the extraction, K5 and the result copies on `stream` and returns a ticket at once;
 * _collect waits for that ticket's work, answers any query the fast match path handed back, writes the rows exactly
 * as aid_query_windows would and hands the ticket back to the engine's pool (also on error). Tickets may be collected
 * in any order; the windows' PCM must stay unchanged until the ticket's work has run (it is read in stream order).
 * Collect every ticket before aid_engine_destroy (the engine frees its pooled tickets, not the outstanding ones). */
typedef struct aid_query_ticket aid_query_ticket;
int aid_query_windows_submit(aid_engine *e, const float *pcm, const int64_t *starts, const int64_t *ends,
                             int32_t n_windows, void *stream, aid_query_ticket **ticket);
int aid_query_windows_collect(aid_engine *e, aid_query_ticket *ticket, aid_match_row *rows, int32_t *nrows);
/* aid_query_pcm in the same two halves (the query coalescer's pipelined batches, replacing the per-request
 * `olaf_c query` processes of fingerprint.py:185-193): HOST PCM is copied to the device in stream order, so the
 * caller keeps it unchanged until it has collected the ticket (with aid_query_windows_collect). */
int aid_query_pcm_submit(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips,
                         int32_t pcm_location, void *stream, aid_query_ticket **ticket);

/* Batched exact lane: replaces app/search/exact.py run_exact_lane's
   sub-window fan-out, the olaf_query calls and the consensus (exact.py:70-124, :132-353) for a
   batch of clips in one call. Clip c = pcm[offsets[c] .. offsets[c+1]) at the engine's sample
   rate (the reference's SAMPLE_RATE, exact.py:58). Clips of <= 5 s are queried as the three
   SUB_WINDOWS (:48-52) and merged by consensus (:220-293), longer clips whole (:296-332);
   candidates below MIN_ALIGNED_HASHES = 8 are dropped and the rest ranked by confidence
   min(h/20, 1), stable, descending (:109-121, :340-353). out: host [n_clips][max_out] rows,
   n_out: host [n_clips]. The metadata lookup (:447-496) stays with the caller. Synchronous. */
typedef struct aid_exact_row {
    uint32_t track;          /* engine track id */
    int32_t aligned_hashes;  /* consensus score */
    double offset_seconds;   /* median reference_start of the track's rows (binary64, as Python) */
    double confidence;       /* min(aligned_hashes / 20, 1) */
} aid_exact_row;
int aid_exact_lane(aid_engine *e, const float *pcm, const int64_t *offsets, int32_t n_clips, int32_t pcm_location,
                   int32_t max_out, aid_exact_row *out, int32_t *n_out, void *stream);
/* The lane's window plan for a clip of n samples (host only, no device): returns the number of
   windows (3 for clips <= 5 s, mode 1; else 1 whole-clip window, mode 0) with sample bounds
   lo[w], len[w] (len 0 = no query, as the reference's empty piece, exact.py:150-160, :374-399). */
int aid_exact_windows(int64_t n, int32_t sample_rate, int64_t *lo, int64_t *len, int32_t *mode);

/* Streaming front end (config 5): interleaved f32 stereo [n_frames][2] -> mono [n_frames] on the
   device, m = (L + R) * 0.5f (the ffmpeg -ac 1 role, decode.py:50-51). Device pointers, stereo
   16-byte and mono 8-byte aligned; asynchronous on `stream`. */
int aid_downmix(aid_engine *e, const float *stereo, int64_t n_frames, float *mono, void *stream);

/* Per-kernel timing with HIP events recorded on the launch stream. */
int aid_profile_enable(aid_engine *e, int32_t on);
/* Which kernels get events while profiling is on: bit k = kernel id k (AID_K_*); default all.
   Each timed launch carries two dispatch-attached events (~5 us of end-of-kernel work per launch on
   MI355X), so a bench can time only the kernels it reports. */
int aid_profile_select(aid_engine *e, uint32_t kernel_mask);
/* ms[AID_K_COUNT] summed device time, launches[AID_K_COUNT]; synchronises; reset != 0 clears. */
int aid_profile_read(aid_engine *e, double *ms, int64_t *launches, int32_t reset);

#ifdef __cplusplus
}
#endif

#endif /* AIDFP_H */
