/*
 * ringpop_amd.h — C ABI of librpamd.so, the MI355X-native engine for ringpop-node's
 * data-parallel core (hash ring, SWIM membership merge + checksum, gossip rounds).
 *
 * Drop-in boundary: these are the entry points a Node N-API addon (or any FFI) binds to
 * replace the reference's in-process hot path. Each function names the reference
 * interface it replaces (paths relative to ringpop v10.9.6). Conventions:
 *   - every function returns 0 on success or a negative status; rp_last_error() gives the
 *     thread-local message. Empty results are NOT errors (reference returns null / []).
 *   - host pointers are borrowed for the duration of the call; *_dev variants take device
 *     pointers and a HIP stream (void*; NULL = the null stream, except rp_wire_decode*_dev,
 *     where NULL = the members handle's own stream) and are stream-ordered. A handle's device
 *     scratch is ordered across streams: a call on another stream than the handle's previous
 *     one first waits for the work queued on that stream. Device-side ordering faults (a
 *     look-back wait that gave up) are reported as RP_EDEVICE at the next host-synchronizing
 *     call on the handle.
 *   - owner ids are interned server ids (stable for the life of a ring); 0xFFFFFFFF = null.
 *   - strings are byte ranges (UTF-8): `bytes` + `off[n+1]` (uint32 offsets) or a fixed
 *     `stride`. Handles are not thread-safe (one HIP stream per handle).
 */
#ifndef RINGPOP_AMD_H
#define RINGPOP_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RP_NULL_ID 0xFFFFFFFFu

/* ------------------------------------------------------------------ common */
const char *rp_last_error(void);
/* Library/ABI version (major<<16 | minor). */
uint32_t rp_version(void);
/* Number of visible HIP devices (0 when none). */
int rp_device_count(int *n);

/* ------------------------------------------------------------------ farmhash32
 * Replaces npm `farmhash` ^0.2.0 hash32 (reference package.json:34), called at
 * lib/ring/index.js:29,55,102,140,146,166 and lib/membership/index.js:65.
 * rp_hash32 is the host C++ implementation (the reference's addon is host C++ too);
 * rp_hash32_batch_dev hashes n device strings (off: n+1 uint64 byte offsets). */
uint32_t rp_hash32(const char *s, size_t len);
int rp_hash32_batch_dev(const uint8_t *d_bytes, const uint64_t *d_off, uint64_t n, uint32_t *d_out,
                        void *stream);
/* farmhash32 of ONE long device string d_bytes[0, len) (the checksum strings of
 * lib/ring/index.js:96-105 and lib/membership/index.js:48-75 are hashed this way): one serial
 * chain fed by producer lanes. d_out[0] = hash (d_out must hold 2 uint32). */
int rp_hash32_long_dev(const uint8_t *d_bytes, uint64_t len, uint32_t *d_out, void *stream);
/* farmhash32 of n long device strings side by side (the membership checksum groups): string b
 * is d_bytes + b * stride; d_meta[4b] = its length + 1 (a builder's piece total), d_meta[4b + 1]
 * = its gate (0: skipped, nothing written); the hash goes to d_meta[4b + 2] and d_meta[4b + 3] =
 * 1. Each string must be readable 12 bytes past its end. 16-B aligned strings at a 16-B multiple
 * stride run kHpStr strings a workgroup (RP_HL_PACK=0: one a workgroup). */
int rp_hash32_long_multi_dev(const uint8_t *d_bytes, uint64_t stride, uint32_t n, uint32_t *d_meta, void *stream);

/* Synthetic key stream: n UUID-v4-format 36-byte keys [k0, k0+n) of `seed`,
 * written at 36-byte stride. */
int rp_gen_uuid_keys_dev(uint32_t seed, uint64_t k0, uint64_t n, uint8_t *d_out, void *stream);

/* ------------------------------------------------------------------ HashRing
 * Replaces lib/ring/index.js HashRing (25-189) and its RBTree (lib/ring/rbtree.js) with a
 * sorted token array in HBM. */
typedef struct rp_ring rp_ring;

/* new HashRing({replicaPoints}) (lib/ring/index.js:25-34); replica_points 0 => 100. */
int rp_ring_create(uint32_t replica_points, int device, rp_ring **out);
int rp_ring_destroy(rp_ring *r);

/* addRemoveServers(serversToAdd, serversToRemove) (lib/ring/index.js:60-94); also the
 * building block of addServer/removeServer (39-48, 124-133). Tokens are farmhash32 of
 * server + String(i) computed on the device, unless add_tokens/rem_tokens (n*R uint32,
 * row j = input server j) carry a caller hashFunc's values (options.hashFunc, :29).
 * *changed_out = ringChanged. The checksum is recomputed on the device when changed. */
int rp_ring_add_remove(rp_ring *r,
                       const char *add_bytes, const uint32_t *add_off, uint32_t n_add,
                       const uint32_t *add_tokens,
                       const char *rem_bytes, const uint32_t *rem_off, uint32_t n_rem,
                       const uint32_t *rem_tokens,
                       int *changed_out);

/* ring.checksum (lib/ring/index.js:33,96-105): farmhash32 of the sorted server names joined
 * by ';'. *is_set = 0 while the reference value would still be null. */
int rp_ring_checksum(rp_ring *r, uint32_t *out, int *is_set);
/* The joined checksum string (for callers with a custom hashFunc): writes up to cap bytes,
 * *len = full length. */
int rp_ring_checksum_string(rp_ring *r, char *buf, uint64_t cap, uint64_t *len);
/* getServerCount (:107-109), rbtree.size, hasServer (:118-120). */
int rp_ring_server_count(rp_ring *r, uint32_t *out);
int rp_ring_token_count(rp_ring *r, uint32_t *out);
int rp_ring_has_server(rp_ring *r, const char *name, uint32_t len, int *out);
/* Interned id of a name (RP_NULL_ID if never seen) and id -> name. */
int rp_ring_server_id(rp_ring *r, const char *name, uint32_t len, uint32_t *id);
const char *rp_ring_owner_name(rp_ring *r, uint32_t id, uint32_t *len);
/* Object.keys(servers) in insertion order (getStats, :111-116): ids_out[cap], *n = count. */
int rp_ring_servers(rp_ring *r, uint32_t *ids_out, uint32_t cap, uint32_t *n);
/* Copy the sorted (token, owner) arrays to host (in-order rbtree walk). */
int rp_ring_dump(rp_ring *r, uint32_t *tokens, uint32_t *owners, uint32_t cap);

/* Batched lookup(key) (:145-154) and lookupN(key, n) (:157-189), host buffers in and out
 * (PCIe-inclusive). Keys: stride > 0 => key i = keys[i*stride .. +stride); else
 * keys[off[i] .. off[i+1]) with uint64 offsets. lookupN output rows have max(n,1) slots,
 * unused = RP_NULL_ID; counts (nullable) = result length per key. */
int rp_ring_lookup(rp_ring *r, const char *keys, const uint64_t *off, uint32_t stride, uint64_t n,
                   uint32_t *owners);
int rp_ring_lookupn(rp_ring *r, const char *keys, const uint64_t *off, uint32_t stride, uint64_t n,
                    int32_t nrep, uint32_t *owners, uint8_t *counts);
/* Low-latency single calls (RingPop.lookup / lookupN per request, index.js:434-471): with
 * idle_ms > 0, a one-key rp_ring_lookup / rp_ring_lookupn / rp_ring_lookupn_hashes (n <= 8; the
 * host hashes the key) is answered by a resident service (eight one-wave workgroups, one an XCD,
 * RP_SVC_WAVES) that polls a pinned, device-mapped request line on a staggered schedule and reads
 * one record of its direct table (built at its first launch after a ring change), instead of a
 * kernel launch and a stream sync per call. The waves exit after idle_ms without a
 * request (and after 30 s in all) and is relaunched by the next call; a ring mutation and every
 * other device call on this ring (batch lookups, grouping, dump) stop it first. Every device
 * call of this library on any other handle stops every resident service as well and keeps new
 * ones from starting until it returns (a resident wave would make its hipFree wait, and its
 * stream may share a hardware queue), so no call of the library waits for a wave to idle out;
 * device work queued outside the library is not covered. idle_ms = 0 (the default) turns it
 * off. */
int rp_ring_service(rp_ring *r, uint32_t idle_ms);
/* Same with precomputed key hashes (hashFunc(key) done by the caller). */
int rp_ring_lookup_hashes(rp_ring *r, const uint32_t *hashes, uint64_t n, uint32_t *owners);
int rp_ring_lookupn_hashes(rp_ring *r, const uint32_t *hashes, uint64_t n, int32_t nrep,
                           uint32_t *owners, uint8_t *counts);
/* Device-resident forms (the hot path): inputs already in HBM, stream-ordered, no sync. */
int rp_ring_lookup_dev(rp_ring *r, const uint8_t *d_keys, const uint64_t *d_off, uint32_t stride,
                       uint64_t n, uint32_t *d_owners, void *stream);
int rp_ring_lookupn_dev(rp_ring *r, const uint8_t *d_keys, const uint64_t *d_off, uint32_t stride,
                        uint64_t n, int32_t nrep, uint32_t *d_owners, uint8_t *d_counts, void *stream);
int rp_ring_lookupn_hashes_dev(rp_ring *r, const uint32_t *d_hashes, uint64_t n, int32_t nrep,
                               uint32_t *d_owners, uint8_t *d_counts, void *stream);

/* Keys grouped by owner: RingPop.handleOrProxyAll's keysByDest = _.groupBy(keys, this.lookup)
 * (index.js:609-667, :616) and RequestProxySend.lookupKeys (lib/request-proxy/send.js:171-179).
 * Every key is looked up (lib/ring/index.js:145-154); on an empty ring every key gets self_id
 * (RingPop.lookup's whoami() fallback, index.js:434-451). Outputs:
 *   dests[0 .. *ndest)        the distinct owners in first-seen order = Object.keys(keysByDest)
 *                             (lookupKeys' result); capacity min(n, server_count + 1)
 *   group_off[0 .. *ndest]    group g holds perm[group_off[g] .. group_off[g+1])
 *   perm[0 .. n)              key indices; each group keeps input order (keysByDest[dest])
 * The _dev form takes device buffers (group_off holding n + 1) and never syncs with the host
 * unless the ring is empty. */
int rp_ring_group_keys_dev(rp_ring *r, const uint8_t *d_keys, const uint64_t *d_off, uint32_t stride, uint64_t n,
                           uint32_t self_id, uint32_t *d_dests, uint32_t *d_group_off, uint32_t *d_perm,
                           uint32_t *d_ndest, void *stream);
int rp_ring_group_keys(rp_ring *r, const char *keys, const uint64_t *off, uint32_t stride, uint64_t n,
                       uint32_t self_id, uint32_t *dests, uint32_t *group_off, uint32_t *perm, uint32_t *ndest);
/* Same with a caller hashFunc's key hashes (options.hashFunc, lib/ring/index.js:29). */
int rp_ring_group_hashes(rp_ring *r, const uint32_t *hashes, uint64_t n, uint32_t self_id, uint32_t *dests,
                         uint32_t *group_off, uint32_t *perm, uint32_t *ndest);

/* ------------------------------------------------------------------ Membership
 * Replaces the hot path of lib/membership/index.js Membership: update (249-324) with the
 * Member.evaluateUpdate rules (lib/membership/member.js:71-202) and computeChecksum /
 * generateChecksumString (48-75, 100-123). Members are interned address ids; status codes
 * 0 alive, 1 suspect, 2 faulty, 3 leave (member.js:204-209). The JS wrapper keeps the
 * Member objects, the members array order (getJoinPosition, 129-131) and the isReady stash
 * (259-265): call update only where the reference would evaluate (ready or isLocal). */
typedef struct rp_members rp_members;

int rp_members_create(uint32_t capacity, int device, rp_members **out);
int rp_members_destroy(rp_members *m);
/* Intern addresses (ids_out[i] for each; existing names keep their id). */
int rp_members_intern(rp_members *m, const char *bytes, const uint32_t *off, uint32_t n, uint32_t *ids_out);
/* whoami(): the local member's id (local override, member.js:155-169). */
int rp_members_set_local(rp_members *m, uint32_t local_id);
/* Membership.update(changes) for k changes (ids, status, incarnation) evaluated in array order
 * with Date.now() = now_ms. applied[i]: 0 not applied, 1 applied, 2 created a new member;
 * new_status/new_inc: the update as applied (local override rewrites it). If anything applied
 * the checksum is recomputed once. Host buffers (all outputs nullable). Incarnations must lie in
 * [-2^60, 2^60) (a JS Number is exact to 2^53; the member table stores 61 bits) and statuses in
 * 0..3, else RP_EINVAL with nothing applied. */
int rp_members_update(rp_members *m, const uint32_t *ids, const uint8_t *status, const int64_t *inc, uint32_t k,
                      int64_t now_ms, uint8_t *applied, uint8_t *new_status, int64_t *new_inc,
                      uint32_t *n_applied);
/* Same, device buffers, stream-ordered, no host synchronization (d_n_applied nullable). An
 * incarnation outside [-2^60, 2^60) is reported as RP_EDEVICE by the handle's next host-
 * synchronizing call. The status / incarnation outputs may be the input arrays themselves (the
 * reference rewrites its update objects in place): the copy is then skipped. */
int rp_members_update_dev(rp_members *m, const uint32_t *d_ids, const uint8_t *d_status, const int64_t *d_inc,
                          uint32_t k, int64_t now_ms, uint8_t *d_applied, uint8_t *d_new_status,
                          int64_t *d_new_inc, uint32_t *d_n_applied, void *stream);
/* The merge partitioned by member id (lib/membership/index.js:249-324 split by id):
 * the same update over device buffers, applied only to the changes whose id lies in [id_lo,
 * id_hi) (whole buckets of 4,096 ids; id_hi may be the capacity). Those changes are evaluated in
 * array order as update_dev would; the outputs (applied, new status / incarnation) of the other
 * changes are left as they were, *d_n_applied counts this range's applied changes, and rows
 * outside the range are not touched. No checksum is computed: a caller holding the table in
 * ranges brings the rows together (rp_members_rows_copy) and calls rp_members_compute_checksum.
 * Always the bucket path (no damp scoring, at most 8M ids); a range past the table folds nothing
 * (*d_n_applied = 0). Stream-ordered, no host sync. */
int rp_members_update_range_dev(rp_members *m, const uint32_t *d_ids, const uint8_t *d_status,
                                const int64_t *d_inc, uint32_t k, int64_t now_ms, uint32_t id_lo, uint32_t id_hi,
                                uint8_t *d_applied, uint8_t *d_new_status, int64_t *d_new_inc,
                                uint32_t *d_n_applied, void *stream);
/* The member rows of ids [id_lo, id_hi) (8 B each: incarnation << 3 | exists << 2 | status) to
 * (into_table = 0) or from (1) a device buffer, on `stream`. */
int rp_members_rows_copy(rp_members *m, void *d_buf, uint32_t id_lo, uint32_t id_hi, int into_table, void *stream);
/* membership.checksum (null until the first applied update: *is_set = 0). */
/* Membership.set (lib/membership/index.js:208-247) over the stash of k changes received while
 * not ready (arrival order; the caller keeps the stash, index.js:259-265):
 * mergeMembershipChangesets (lib/membership/merge.js:22-51: the local member skipped, the
 * strictly greatest incarnation per address wins, the first one on ties), then every picked
 * change is set verbatim (existing members overwritten, unknown addresses created), then the
 * checksum is computed once. pick (k entries) receives the indices of the picked changes in
 * first-seen address order (the order the caller appends new Member objects in), npick their
 * count. The _dev form takes device buffers and never syncs with the host. */
int rp_members_set(rp_members *m, const uint32_t *ids, const uint8_t *status, const int64_t *inc, uint32_t k,
                   uint32_t *pick, uint32_t *npick);
int rp_members_set_dev(rp_members *m, const uint32_t *d_ids, const uint8_t *d_status, const int64_t *d_inc,
                       uint32_t k, uint32_t *d_pick, uint32_t *d_npick, void *stream);
int rp_members_checksum(rp_members *m, uint32_t *out, int *is_set);
/* computeChecksum() unconditionally. */
int rp_members_compute_checksum(rp_members *m);
/* defer != 0: update no longer recomputes the checksum after each batch (the reference does,
 * index.js:306-309); a caller folding many batches calls rp_members_compute_checksum once at the
 * end. Default off. */
int rp_members_defer_checksum(rp_members *m, int defer);
/* Batch-strided checksums over replicas (§8e membership merge on G GPUs: every replica folds
 * every batch, so each holds the whole table; the checksum strings and their serial farmhash
 * chains, index.js:48-75 / 306-309, are divided among the replicas). From this call on, update
 * batch b (counting update calls with k > 0 from 0) builds and hashes its checksum only when
 * b % nshards == shard. With history_cap > 0 each such batch's {checksum, applied-anything} is
 * recorded in order (at most history_cap of them; rp_members_checksum_history reads them). A
 * batch that applied nothing leaves the reference's checksum unchanged: a reader carries the
 * previous batch's value forward. nshards = 1, shard = 0 restores the default. */
int rp_members_checksum_shard(rp_members *m, uint32_t nshards, uint32_t shard, uint32_t history_cap);
/* The recorded per-batch checksums (this shard's batches, in batch order): hash[i], applied[i]
 * (0: the batch applied nothing; hash[i] is then 0), up to cap; *n = entries recorded. */
int rp_members_checksum_history(rp_members *m, uint32_t *hash, uint8_t *applied, uint32_t cap, uint32_t *n);
/* Drop the first `count` recorded entries (after reading them), so a long-running replica keeps
 * recording: update refuses a batch with RP_ESTATE, before applying anything, when its entry
 * would not fit history_cap. */
int rp_members_checksum_history_drain(rp_members *m, uint32_t count);
/* generateChecksumString() (writes up to cap bytes; *len = full length). */
int rp_members_checksum_string(rp_members *m, char *buf, uint64_t cap, uint64_t *len);
/* Member table by id (exists/status/incarnation), cap entries. */
int rp_members_dump(rp_members *m, uint8_t *exists, uint8_t *status, int64_t *inc, uint32_t cap);
int rp_members_count(rp_members *m, uint32_t *n_names);

/* ---- flap-damping scores ----
 * Member.dampScore / lastUpdateDampScore / lastUpdateTimestamp (lib/membership/member.js:28-41)
 * kept on the device by member id. Once configured, every update() applies _applyUpdatePenalty
 * (member.js:98-107, 133-153: decay, + penalty, clamp, suppress-limit check) to each applied
 * update of another member at now_ms, stamps lastUpdateTimestamp on every applied update, and
 * gives created members (update() or set()) the initial score; rp_members_damp_decay is
 * Membership._decayMembersDampScore (lib/membership/index.js:374-383) over every member. The
 * fields mirror config.js:60-71; the defaults are {1, 0, 0, 10000, 500, 5000, 60}. The decay
 * factor is V8's Math.pow (fdlibm) restated bit for bit. */
typedef struct rp_damp_config {
    int enabled;            /* dampScoringEnabled: penalize applied updates */
    double initial;         /* dampScoringInitial */
    double min;             /* dampScoringMin */
    double max;             /* dampScoringMax */
    double penalty;         /* dampScoringPenalty */
    double suppress_limit;  /* dampScoringSuppressLimit */
    double half_life;       /* dampScoringHalfLife, seconds (> 0) */
} rp_damp_config;

/* Turn tracking on (first call: every id starts at `initial`, null timestamp) or change the
 * config. Call it where the reference constructs Membership (initMembership, index.js:399-418). */
int rp_members_damp_configure(rp_members *m, const rp_damp_config *cfg);
/* The last update batch, per change in batch order: the member's dampScore after the change and
 * whether 'suppressLimitExceeded' fired (member.js:141-152). k <= that batch's size. */
int rp_members_damp_last(rp_members *m, double *score, uint8_t *exceeded, uint32_t k);
/* The decayer tick at Date.now() = now_ms (host form syncs; _dev is stream-ordered). */
int rp_members_damp_decay(rp_members *m, int64_t now_ms);
int rp_members_damp_decay_dev(rp_members *m, int64_t now_ms, void *stream);
/* Per id (cap entries, nullable outputs): dampScore, lastUpdateDampScore, lastUpdateTimestamp
 * (0 = null). */
int rp_members_damp_dump(rp_members *m, double *score, double *last_score, int64_t *last_ts, uint32_t cap);

/* ------------------------------------------------------------------ Gossip wire bodies
 * Change records as the JSON text ringpop sends (addresses are ids interned in the members
 * handle m). Replaces the per-message JSON.stringify / safeParse of:
 *   issueAs record  {id, source, sourceIncarnationNumber, address, status, incarnationNumber}
 *                   (lib/gossip/dissemination.js:163-170)                                form 0
 *   fullSync record {source, address, status, incarnationNumber} (dissemination.js:64-73)  form 1
 * and the bodies around them (RP_WIRE_BODY_*):
 *   ARRAY             the bare changes array
 *   PING              {checksum, changes, source, sourceIncarnationNumber}  lib/gossip/ping-sender.js:71-76
 *   PING_RESPONSE     {changes}                                              server/protocol/ping.js:45-48
 *   PINGREQ           {checksum, changes, source, sourceIncarnationNumber, target}
 *                                                                    lib/gossip/ping-req-sender.js:75-81
 *   PINGREQ_RESPONSE  {changes, pingStatus, target}                     server/protocol/ping-req.js:61-65
 *   JOIN_RESPONSE     {app, coordinator, membership, membershipChecksum}  server/protocol/join.js:128-133
 *                     (membership = the fullSync records; coordinator = the source column,
 *                     membershipChecksum = the checksum column, app = one string for the batch)
 * JSON.stringify leaves an undefined member out; per record: an ids row whose first byte is NUL,
 * a src of RP_NULL_ID, a src_inc of INT64_MIN (or a null column) are absent and not written.
 * Message j holds records [msg_rec_off[j], msg_rec_off[j+1]): msg_rec_off[0] = 0, not
 * decreasing, msg_rec_off[n_msgs] = n_rec. Every id and offset is validated on the device before
 * anything is written (RP_EINVAL otherwise). Encode writes d_out_off[0..n_msgs] (byte offsets);
 * with d_out null only the offsets are computed (size query). Synchronous. */
enum {
    RP_WIRE_BODY_ARRAY = 0,
    RP_WIRE_BODY_PING = 1,
    RP_WIRE_BODY_PING_RESPONSE = 2,
    RP_WIRE_BODY_PINGREQ = 3,
    RP_WIRE_BODY_PINGREQ_RESPONSE = 4,
    RP_WIRE_BODY_JOIN_RESPONSE = 5
};
typedef struct rp_wire_records {  /* n_rec entries each */
    const uint32_t *addr, *src;     /* member ids (src: RP_NULL_ID = absent) */
    const uint8_t *status;          /* 0 alive 1 suspect 2 faulty 3 leave */
    const int64_t *inc, *src_inc;   /* incarnationNumber; sourceIncarnationNumber (INT64_MIN / null = absent) */
    const uint8_t *ids;             /* 36-byte uuids per record, nullable */
} rp_wire_records;
typedef struct rp_wire_headers {  /* n_msgs entries each, as the body needs them */
    const uint32_t *checksum;       /* PING, PINGREQ: checksum; JOIN_RESPONSE: membershipChecksum */
    const uint32_t *source;         /* PING, PINGREQ: source; JOIN_RESPONSE: coordinator */
    const int64_t *source_inc;      /* PING, PINGREQ: sourceIncarnationNumber */
    const uint32_t *target;         /* PINGREQ, PINGREQ_RESPONSE: target */
    const uint8_t *ping_status;     /* PINGREQ_RESPONSE: pingStatus (0 / 1) */
    const char *app;                /* JOIN_RESPONSE: app (host string, app_len bytes, no escapes) */
    uint32_t app_len;
} rp_wire_headers;
int rp_wire_encode_dev(rp_members *m, uint32_t n_msgs, const uint32_t *d_msg_rec_off, uint64_t n_rec,
                       const rp_wire_records *d_recs, int form, int body, const rp_wire_headers *d_hdr,
                       uint8_t *d_out, uint64_t *d_out_off, void *stream);
/* Host-buffer form (staged through the handle's device; PCIe-bound; ids checked on the host):
 * out NULL = size query (out_off filled); otherwise cap >= out_off[n_msgs]. */
int rp_wire_encode(rp_members *m, uint32_t n_msgs, const uint32_t *msg_rec_off, const rp_wire_records *recs,
                   int form, int body, const rp_wire_headers *hdr, uint8_t *out, uint64_t cap, uint64_t *out_off);

/* Decode n_msgs JSON texts buf[msg_off[j] .. msg_off[j+1]) — a changes array, or a body object
 * whose `changes` (join response: `membership`) member is one; any key order, JSON whitespace,
 * unknown members skipped (server/protocol/ping.js:27-36 reads the same members). msg_rec_off[0..n_msgs]
 * gets record offsets (total in [n_msgs]); records beyond rec_cap are counted, not written. Per
 * record: address id (RP_NULL_ID if not interned; addr_off / addr_len give its bytes), source id
 * (RP_NULL_ID: absent or not interned), status, incarnationNumber, sourceIncarnationNumber
 * (INT64_MIN if absent), byte offset of `id` (~0 if absent). Per message: checksum /
 * membershipChecksum, source / coordinator, sourceIncarnationNumber, target, pingStatus (0xFF if
 * absent); err[j] = 0, or 1 + the failing byte's offset in message j (its records are then
 * dropped). Strings with escapes and non-integral numbers are rejected (addresses and uuids
 * never hold one). Every column except addr / status / inc is nullable. */
typedef struct rp_wire_records_out {
    uint32_t *addr, *src;
    uint8_t *status;
    int64_t *inc, *src_inc;
    uint64_t *id_off, *addr_off;
    uint32_t *addr_len;
} rp_wire_records_out;
typedef struct rp_wire_headers_out {
    uint32_t *checksum, *source;
    int64_t *source_inc;
    uint32_t *target;
    uint8_t *ping_status;
} rp_wire_headers_out;
int rp_wire_decode_dev(rp_members *m, const uint8_t *d_buf, const uint64_t *d_msg_off, uint32_t n_msgs,
                       uint32_t *d_msg_rec_off, uint32_t rec_cap, const rp_wire_records_out *d_recs,
                       const rp_wire_headers_out *d_hdr, uint64_t *d_err, void *stream);
int rp_wire_decode(rp_members *m, const char *buf, const uint64_t *msg_off, uint32_t n_msgs, uint32_t *msg_rec_off,
                   uint32_t rec_cap, const rp_wire_records_out *recs, const rp_wire_headers_out *hdr, uint64_t *err);

/* The first round's column-list forms of the same codec (bodies 0..2). */
int rp_wire_encode_changes_dev(rp_members *m, uint32_t n_msgs, const uint32_t *d_msg_rec_off, uint64_t n_rec,
                               const uint32_t *d_addr, const uint32_t *d_src, const uint8_t *d_status,
                               const int64_t *d_inc, const int64_t *d_src_inc, const uint8_t *d_ids, int form,
                               int body, const uint32_t *d_msg_checksum, const uint32_t *d_msg_source,
                               const int64_t *d_msg_source_inc, uint8_t *d_out, uint64_t *d_out_off, void *stream);
int rp_wire_encode_changes(rp_members *m, uint32_t n_msgs, const uint32_t *msg_rec_off, const uint32_t *addr,
                           const uint32_t *src, const uint8_t *status, const int64_t *inc, const int64_t *src_inc,
                           const uint8_t *ids, int form, int body, const uint32_t *msg_checksum,
                           const uint32_t *msg_source, const int64_t *msg_source_inc, uint8_t *out, uint64_t cap,
                           uint64_t *out_off);
int rp_wire_decode_changes_dev(rp_members *m, const uint8_t *d_buf, const uint64_t *d_msg_off, uint32_t n_msgs,
                               uint32_t *d_msg_rec_off, uint32_t rec_cap, uint32_t *d_addr, uint32_t *d_src,
                               uint8_t *d_status, int64_t *d_inc, int64_t *d_src_inc, uint64_t *d_id_off,
                               uint64_t *d_addr_off, uint32_t *d_addr_len, uint64_t *d_err,
                               uint32_t *d_msg_checksum, uint32_t *d_msg_source, int64_t *d_msg_source_inc,
                               void *stream);
int rp_wire_decode_changes(rp_members *m, const char *buf, const uint64_t *msg_off, uint32_t n_msgs,
                           uint32_t *msg_rec_off, uint32_t rec_cap, uint32_t *addr, uint32_t *src, uint8_t *status,
                           int64_t *inc, int64_t *src_inc, uint64_t *err);

/* ------------------------------------------------------------------ Gossip simulator
 * N full ringpop nodes (every node: membership view, dissemination buffer, ring membership,
 * iterator, suspicion timers; lib/membership, lib/gossip, lib/ring, lib/on_membership_event.js)
 * advanced in the deterministic round model of DESIGN.md §SWIM round model: ping / ping-req
 * exchange, piggyback counters with maxPiggybackCount, suspect->faulty timers. No reference
 * counterpart (the reference is one view per process). names/off: N member addresses;
 * inc0[N]: initial incarnations (every view starts identical, all alive); dead[N]: members
 * killed before round 0. seed: Philox seed of the iterator shuffles and ping-req samples;
 * suspicion_rounds: 5000 ms / 200 ms = 25 by default; now0: Date.now() at round 0. */
typedef struct rp_sim rp_sim;

int rp_sim_create(uint32_t n, const char *names, const uint32_t *off, const int64_t *inc0, const uint8_t *dead,
                  uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, rp_sim **out);
int rp_sim_destroy(rp_sim *s);
/* Advance `rounds` rounds (synchronous) / enqueue them (asynchronous, rp_sim_sync waits). */
int rp_sim_step(rp_sim *s, uint32_t rounds);
int rp_sim_step_async(rp_sim *s, uint32_t rounds);
int rp_sim_sync(rp_sim *s);
int rp_sim_round(rp_sim *s, int64_t *out);
/* Every node's membership checksum (0 for killed nodes). */
int rp_sim_checksums(rp_sim *s, uint32_t *out);
/* Node v's view: status[N], incarnation[N] (nullable). */
int rp_sim_view(rp_sim *s, uint32_t v, uint8_t *status, int64_t *inc);
/* Convergence (scenario-runner.js:152-170): all live checksums equal and every killed member
 * faulty in every live view. */
int rp_sim_converged(rp_sim *s, int *out);
/* pings, ping-reqs, full syncs, applied updates since creation. */
int rp_sim_stats(rp_sim *s, uint64_t *out4);

/* ---- Sharded simulator (C5): a handle owns the nodes [bounds[shard], bounds[shard+1]) of a
 * partition of [0, n) into nshards contiguous ranges (bounds NULL = equal ranges); its views
 * still cover all n members. A round is five stages (rp_sim_stage 0..4) separated by four
 * message exchanges: after stage k < 4 the outbox holds this shard's messages grouped by
 * destination shard (rp_sim_outbox: per-destination message / record counts and ONE device
 * buffer holding, for each destination in shard order, a segment of its 40-byte headers then
 * its 24-byte records); before stage k + 1 the caller fills the inbox (rp_sim_inbox sizes it for
 * the per-source counts and returns its device buffer) with every source's segment for this
 * shard, in source-shard order — one all-to-all-v moves the bytes as they lie. The buffers are
 * owned by the handle and valid until its next stage. Neither call waits for the device (round
 * 6): the counts are on the host when rp_sim_stage returns, but the outbox bytes are written, and
 * the inbox is still read by the previous stage, on the handle's stream. Before reading the
 * outbox or writing the inbox the caller orders itself after that stream with
 * rp_sim_order_stream (a device stream waits on the device; NULL: the host waits). rp_sim_exchange_local does the
 * exchange for handles of one process; across processes the host moves the bytes (RCCL
 * all-to-all-v; ringpop-node_amd DistGossipSim). Checksums / views / stats are per shard
 * (checksums: the shard's nodes in id order); convergence reduces rp_sim_converged_local
 * {live nodes, min checksum, max checksum, killed-not-faulty flag} over the shards. */
int rp_sim_create_shard(uint32_t n, const char *names, const uint32_t *off, const int64_t *inc0, const uint8_t *dead,
                        uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device, const uint32_t *bounds,
                        uint32_t nshards, uint32_t shard, rp_sim **out);
int rp_sim_shard_info(rp_sim *s, uint32_t *v0, uint32_t *nl, uint32_t *nshards, uint32_t *shard);
int rp_sim_stage(rp_sim *s, int stage);
int rp_sim_outbox(rp_sim *s, uint64_t *nmsg, uint64_t *nrec, void **buf);
int rp_sim_inbox(rp_sim *s, const uint64_t *nmsg, const uint64_t *nrec, void **buf);
/* The handle's next stage waits (on the device, no host sync) for the work queued so far on
 * `stream`: a caller that moved the inbox bytes with a collective on its own stream (RCCL on
 * torch's stream) orders the import after it this way. */
int rp_sim_wait_stream(rp_sim *s, void *stream);
/* The converse: `stream` waits (on the device) for the work queued so far on the handle's stream;
 * stream NULL: the host waits for it. */
int rp_sim_order_stream(rp_sim *s, void *stream);
int rp_sim_exchange_local(rp_sim *const *shards, uint32_t nshards);
int rp_sim_converged_local(rp_sim *s, uint32_t *out4);
/* JOIN events on a sharded simulator (a joiner reads its responders' views, which other shards
 * may hold). Before rp_sim_stage(s, 0) of every round, on every shard, repeat until *has == 0:
 * rp_sim_join_export applies the round's events up to its next join, runs the join handler of
 * the responders this shard owns and returns a device buffer of *bytes bytes holding their
 * rows (zeros elsewhere; every byte has exactly one writing shard). The caller combines the
 * shards' buffers into each shard's own buffer by a byte-wise sum (an RCCL / gloo all-reduce of
 * uint8, or rp_sim_join_exchange_local for handles in one process), then calls
 * rp_sim_join_import, which builds the joiner's view on its shard. (Replaces the responders'
 * join handler + the joiner's mergeJoinResponses / set(): server/protocol/join.js:126,
 * join-response-merge.js:40-56, membership/index.js:208-247.) */
int rp_sim_join_export(rp_sim *s, int *has, void **buf, uint64_t *bytes);
int rp_sim_join_import(rp_sim *s);
int rp_sim_join_exchange_local(rp_sim *const *shards, uint32_t nshards);

/* ---- Scenarios. Events run before phase A of their round, in the order given:
 *   RP_SIM_KILL    the node goes down (crash / SIGSTOP, scripts/tick-cluster.js:417-470): it
 *                  neither acts nor answers; its state is kept
 *   RP_SIM_REVIVE  it comes back with that state (SIGCONT)
 *   RP_SIM_LEAVE   the admin leave (server/admin/member.js:70-98): makeLeave(whoami, own
 *                  incarnation) (lib/membership/index.js:191-195), as the convergence scenarios
 *                  send it (benchmarks/convergence-time/scenarios/); its LocalMemberLeaveEvent
 *                  stops the node's gossip loop and suspicion (on_membership_event.js:32-40). A
 *                  node that is down, or left already, ignores it.
 *   RP_SIM_JOIN    a fresh process for the node bootstraps into the running cluster
 *                  (index.js:240-322): makeAlive(self, Date.now()); three live nodes (JOIN
 *                  Philox stream over the live nodes in id order) answer the join
 *                  (server/protocol/join.js:126-133: makeAlive(joiner), fullSync);
 *                  mergeJoinResponses (join-response-merge.js:40-56) is stashed and set()
 *                  (index.js:208-247) builds the view, the set handler
 *                  (on_membership_event.js:42-67) fills the ring and the suspicion timers; the
 *                  dissemination is cleared as at bootstrap, then gossip.start shuffles. Needs an
 *                  unsharded handle and one live node besides the joiner.
 * Convergence then reads: every node that is up and has not left holds the same checksum, each
 * member that left is `leave` and each other member that is down `faulty` in those views.
 * dead[] = down from the start (never started gossip; gossip/index.js:97 never shuffled). */
typedef struct rp_sim_event {
    uint32_t round, kind, node, reserved;
} rp_sim_event;
enum { RP_SIM_KILL = 0, RP_SIM_REVIVE = 1, RP_SIM_LEAVE = 2, RP_SIM_JOIN = 3 };
int rp_sim_create_scenario(uint32_t n, const char *names, const uint32_t *off, const int64_t *inc0,
                           const uint8_t *dead, uint32_t seed, uint32_t suspicion_rounds, int64_t now0, int device,
                           const uint32_t *bounds, uint32_t nshards, uint32_t shard, const rp_sim_event *events,
                           uint32_t n_events, rp_sim **out);
/* Every local node's dissemination.maxPiggybackCount (dissemination.js:38-55), [shard nodes]. */
int rp_sim_piggyback(rp_sim *s, uint32_t *out);
/* Traffic since creation: {pings, ping-reqs, full syncs, applied updates, messages sent, change
 * records sent, views hashed, bytes of the all-alive checksum string (a view's string length
 * within a few bytes per deviated member)}. */
int rp_sim_counters(rp_sim *s, uint64_t *out8);

/* Stream-ordered copy between any host / device buffers (hipMemcpyDefault); NULL stream =
 * synchronous. Used by hosts that move sharded-simulator messages. */
int rp_copy(void *dst, const void *src, uint64_t bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif
