/*
 * minbft_gpu.h -- C-ABI of the MI355X batch message authenticator for MinBFT.
 *
 * This is the drop-in boundary for MinBFT's message-authentication hot path.
 * Every entry point takes plain pointers and sizes, returns an integer code,
 * never throws, and never retains caller buffers after returning.
 *
 * What each entry point replaces in the reference (hyperledger-labs/minbft,
 * paths relative to the repository root):
 *
 *   mbft_ctx_create / mbft_add_role / mbft_set_public_key_* / mbft_enable_usig
 *       sample/authentication/authenticator.go:43-116 (New / NewWithSGXUSIG /
 *       NewWithUSIG / new: role -> scheme wiring) and
 *       sample/authentication/keymanager.go:179-227,352-366
 *       (LoadSimpleKeyStore, ecdsaKeySpec.parsePublicKey: x509 PKIX decode
 *       with on-curve validation).  Keys are validated and their comb tables
 *       precomputed on the GPU once (the replica set is static).
 *
 *   mbft_verify_message_authen_tag
 *       api/api.go:133-144 Authenticator.VerifyMessageAuthenTag, implemented
 *       by sample/authentication/authenticator.go:121-134 with the schemes
 *       sample/authentication/crypto.go:79-89,113-126 (ECDSA roles: digest =
 *       msg || SHA256(""), DER decode, crypto/ecdsa.Verify) and
 *       crypto.go:186-239 + usig/sgx/sgx-usig.go:81-101 +
 *       usig/sgx/usig-enclave.go:198-229 (USIG role: UI decode, epoch
 *       capture, SHA256(SHA256(msg)||epoch_le||counter_le), strict DER).
 *       Returns an mbft_status (>= 0) or an mbft_err (< 0).  MBFT_ACCEPT is
 *       Go's nil; MBFT_MALFORMED_DER in an ECDSA role is where Go panics
 *       (crypto.go:82-84); every other status is a Go error.
 *
 *   mbft_verify_batch
 *       NEW batch entry point (north_star item 1/2): n independent calls of
 *       the above, verified together on the GPU.  Results are exactly those
 *       of calling mbft_verify_message_authen_tag on items[0..n) in order:
 *       the USIG epoch capture (crypto.go:219-236) is replayed on the host in
 *       item order after the GPU has checked every signature.
 *
 *   mbft_generate_message_authen_tag
 *       api/api.go:143 GenerateMessageAuthenTag for the ECDSA roles
 *       (crypto.go:63-76,113-116: sign SHA256("")-suffixed digest, DER).
 *       The nonce is deterministic (RFC 6979-style) instead of crypto/rand;
 *       tags verify identically.  USIG generation stays in the SGX enclave.
 *       NOT CONSTANT-TIME (the GPU signer, k_sign, gathers comb entries at
 *       addresses set by the nonce's digits): for tests and synthetic load
 *       only.  A production signer keeps the reference's CPU path (Go's
 *       constant-time P-256, crypto.go:63-76), as the Go binding does
 *       (go/gpuauth: GenerateMessageAuthenTag never calls the GPU).
 *
 *   mbft_verify_prehashed / mbft_verify_prehashed_device
 *       Go crypto/ecdsa.Verify(pub, hash, r, s) as called at
 *       sample/authentication/crypto.go:86 and
 *       usig/sgx/usig-enclave.go:224, for a batch of already-decoded
 *       (e, r, s, key slot) items.  The _device variant takes device
 *       pointers and an hipStream_t (as void*) and is what bench.py times.
 *
 *   mbft_der_parse_sig
 *       encoding/asn1.Unmarshal(sig, &struct{R, S *big.Int}) as used at
 *       crypto.go:81 and usig-enclave.go:217 (host-only, no GPU needed).
 */
#ifndef MINBFT_GPU_H
#define MINBFT_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-item verification outcome (also the value returned by
 * mbft_verify_message_authen_tag). */
enum mbft_status {
  MBFT_ACCEPT = 0,         /* Go: nil */
  MBFT_REJECT_SIG = 1,     /* ecdsa.Verify false: r/s range, infinity, x mismatch */
  MBFT_MALFORMED_DER = 2,  /* asn1.Unmarshal error (ECDSA roles: Go panics) */
  MBFT_DER_TRAILING = 3,   /* USIG: "extra bytes in USIG signature" */
  MBFT_UNKNOWN_KEY = 4,    /* known role, no key for this id (pk == nil) */
  MBFT_BAD_KEY = 5,        /* key slot invalid (never reachable from Go) */
  MBFT_BAD_UI = 6,         /* USIG tag shorter than 8 bytes (usig.go:75-80) */
  MBFT_BAD_CERT = 7,       /* USIG cert shorter than 8 bytes (sgx-usig.go:159-168) */
  MBFT_ZERO_COUNTER = 8,   /* core/usig-ui.go:65-67 (core-level check) */
  MBFT_EPOCH_MISMATCH = 9, /* sgx-usig.go:92-94 */
  MBFT_UNKNOWN_ROLE = 10   /* keymanager.go:100, authenticator.go:126-129 */
};

/* Return codes of API calls (negative). */
enum mbft_err {
  MBFT_OK = 0,
  MBFT_ERR_ARG = -1,
  MBFT_ERR_HIP = -2,
  MBFT_ERR_NOMEM = -3,
  MBFT_ERR_KEY = -4,     /* invalid / off-curve public key (x509 parse error) */
  MBFT_ERR_STATE = -5,   /* e.g. signing without a private key */
  MBFT_ERR_NODEV = -6    /* no usable GPU */
};

/* api/api.go:98-115 AuthenticationRole */
enum mbft_role { MBFT_ROLE_REPLICA = 1, MBFT_ROLE_USIG = 2, MBFT_ROLE_CLIENT = 3 };

typedef struct mbft_ctx mbft_ctx;

/* One authenticator call for mbft_verify_batch. */
typedef struct mbft_item {
  uint32_t role;
  uint32_t id;
  const uint8_t* msg;
  size_t msg_len;
  const uint8_t* tag;
  size_t tag_len;
} mbft_item;

int mbft_version(void);
int mbft_device_count(void);

/* Context = one authenticator.  Created on one GPU (builds the generator
 * comb table there); mbft_ctx_add_device adds an engine on another GPU of
 * the node (or the same one: more streams), which receives replicas of the
 * generator and every key table, now and for keys registered later.  The
 * host-buffer entry points (mbft_verify_batch, mbft_verify_message_authen_tag,
 * mbft_verify_prehashed, mbft_validate_messages) then split each batch into
 * contiguous shards of at least mbft_set_shard_min items (default 32768),
 * one host thread, HIP stream and device per engine, with no collective:
 * only each shard's status bytes come back, in index order, and the USIG
 * epoch replay runs afterwards on the host.  The *_device entry points run
 * on the creating device only.  mbft_ctx_devices returns the engine count
 * and fills devices[0..cap).  (Multi-process, one GPU per process, is the
 * other multi-GPU model: bench.py and DESIGN.md §7.) */
int mbft_ctx_create(int device, mbft_ctx** out);
void mbft_ctx_destroy(mbft_ctx* ctx);
const char* mbft_last_error(const mbft_ctx* ctx);
int mbft_ctx_add_device(mbft_ctx* ctx, int device);
int mbft_ctx_devices(const mbft_ctx* ctx, int* devices, int cap);
int mbft_set_shard_min(mbft_ctx* ctx, size_t items);

/* Key store.  A role exists once declared (even with no keys).  Public keys
 * are 91-byte PKIX DER (keymanager.go:352-366) or raw 64-byte X||Y. */
int mbft_add_role(mbft_ctx* ctx, uint32_t role);
int mbft_set_public_key_pkix(mbft_ctx* ctx, uint32_t role, uint32_t id, const uint8_t* pkix,
                             size_t len);
int mbft_set_public_key_xy(mbft_ctx* ctx, uint32_t role, uint32_t id, const uint8_t xy[64]);
/* Registers raw points without the role/id mapping; out_slots receive key
 * slots for mbft_verify_prehashed*.  valid_out[i] = 1 if on-curve. */
int mbft_register_points(mbft_ctx* ctx, const uint8_t* xy64, size_t n, uint32_t* out_slots,
                         uint8_t* valid_out);
/* Drops every key: all (role, id) -> key mappings, all slots and their comb
 * tables, and the USIG epoch state; declared roles stay.  The tables' device
 * blocks are kept for reuse by the next registrations (re-mapping 129 GiB
 * takes seconds) and released when the generator table is rebuilt, when an
 * allocation would otherwise fail, and at destroy.  Equivalent to
 * building the authenticator again over a new key store
 * (keymanager.go:179-227 LoadSimpleKeyStore + authenticator.go:88-116).
 * Waits for in-flight work. */
int mbft_clear_keys(mbft_ctx* ctx);
/* Slot of (role, id), or MBFT_ERR_KEY if absent. */
int mbft_key_slot(const mbft_ctx* ctx, uint32_t role, uint32_t id);
/* Comb windows.  Signed digits: a window of W bits costs
 * ceil(256/W) table entries per scalar and about ceil(256/W) x 2^(W-1) x
 * 64 B of HBM per table:
 *   W =  8: 32 entries, 0.25 MiB      W = 24: 11 entries, 5.0 GiB
 *   W = 16: 16 entries, 34 MiB        W = 26: 10 entries, 18.3 GiB
 *   W = 22: 12 entries, 1.4 GiB       W = 29:  9 entries, 129 GiB
 * (the last window's table is cut to the digits a 256-bit scalar reaches).
 * mbft_set_key_window sets the window for keys registered AFTER the call
 * (default 16); a single static signer fits at W = 29 next to a W = 29
 * generator table (258 GiB of 288), a 33-replica set at W = 24, a very
 * large client set at W = 8.  mbft_set_generator_window rebuilds the shared
 * generator table (default 16); it waits for in-flight work.
 * Both accept 4 <= W <= 29; MBFT_ERR_NOMEM if the table does not fit. */
int mbft_set_key_window(mbft_ctx* ctx, int wbits);
int mbft_set_generator_window(mbft_ctx* ctx, int wbits);
int mbft_get_windows(const mbft_ctx* ctx, int* g_wbits, int* q_wbits);
/* USIG scheme present (authenticator.go:102-110: absent without a USIG). */
int mbft_enable_usig(mbft_ctx* ctx, int enabled);
/* Private key for GenerateMessageAuthenTag in an ECDSA role. */
int mbft_set_private_key(mbft_ctx* ctx, uint32_t role, const uint8_t d[32]);

/* api.Authenticator */
int mbft_verify_message_authen_tag(mbft_ctx* ctx, uint32_t role, uint32_t id,
                                   const uint8_t* msg, size_t msg_len, const uint8_t* tag,
                                   size_t tag_len);
int mbft_verify_batch(mbft_ctx* ctx, const mbft_item* items, size_t n, uint8_t* status_out);
/* Coalescing of concurrent single calls (new; the reference's ECDSA scheme
 * is called from many goroutines at once, api/api.go:132).  When enabled,
 * mbft_verify_message_authen_tag calls that arrive while the batch slots are
 * busy are queued and verified together as the next batch (group commit):
 * one batch at a time (mbft_set_coalescing_slots: up to that many), the
 * first queued caller without a slot leads the next one, every caller gets
 * its own status, and each batch keeps the queue's order (the USIG epoch step
 * runs in that order --
 * concurrent callers have no order of their own, as under the reference's
 * mutex, crypto.go:215-218).  max_wait_us > 0 also lets a leader wait that
 * long for company when it would otherwise run alone; 0 adds no latency.
 * max_batch caps a batch (0: no cap).  Default: disabled (each call is its
 * own GPU round trip). */
int mbft_set_coalescing(mbft_ctx* ctx, int enabled, uint32_t max_wait_us, uint32_t max_batch);
/* Coalesced batches in flight at once (new): 1..64, default 1; at most the
 * mbft_set_concurrency lanes are used (each batch runs on a lane). */
int mbft_set_coalescing_slots(mbft_ctx* ctx, int slots);
/* The resident single-call verifier (new; replaces, for
 * mbft_verify_message_authen_tag, the per-call kernel launch behind
 * api/api.go:133-144 / sample/authentication/authenticator.go:121-134).
 * slots 1..64: a verify kernel stays on the GPU while calls keep arriving:
 * mailbox slots in host-mapped memory served by a pool of 256-thread
 * workgroups (2 per slot up to MBFT_RESIDENT_SERVERS, default 16); a call
 * takes a free slot, runs its host part (role, DER, digest, key, s^-1),
 * posts the item and sleeps through its expected GPU time, then waits on its
 * done words -- no launch, no stream synchronize, and concurrent callers (up
 * to `slots`) never wait for each other's batch.  The kernel leaves after MBFT_RESIDENT_IDLE_US (default
 * 2000) without a call or MBFT_RESIDENT_LIFE_MS (default 200) after its
 * start, and the next call relaunches it (a relaunch under batch load waits
 * for CUs: at 20 ms a trickle's p99 was ~200 us, at 200 ms 32-51 us).  A
 * device-wide synchronize of the application waits for the live generation;
 * the library's own batch paths make none.  Calls past `slots` at once take
 * the coalescer / batch path.  Statuses, USIG epoch step and errors are those
 * of the other paths.  0 (default) turns it off; waits for calls in flight. */
int mbft_set_resident(mbft_ctx* ctx, int slots);
/* out[6]: slots, calls served, kernel launches, calls that found every slot
 * taken, relaunches found by a stream query, 1 if the kernel's stream has
 * its own hardware queue (the lowest stream priority, which no other stream
 * of the library uses; or CU-masked with MBFT_RESIDENT_CUMASK=1). */
int mbft_resident_stats(mbft_ctx* ctx, double out[6]);
/* out[5] (new, round 6): the caller-side wait of resident calls -- sleeps
 * taken, sleeps that woke after the items were done, the current estimates
 * (ns) of a lone item's post -> done time and of a sleep's wake-up delay,
 * and 1 if the wait sleeps (MBFT_RESIDENT_SLEEP, default 1) or 0 if it spins.
 * The CPU a call costs its caller is its host part, the join, the wake-up and
 * the last spin, not the GPU time (the reference verifies on the calling
 * goroutine's CPU, api/api.go:132, sample/authentication/crypto.go:79-89). */
int mbft_resident_wait_stats(mbft_ctx* ctx, double out[5]);
/* Test hook (new, round 6): host threads the library has started so far
 * (worker pools, one shard thread per engine).  A batch on a multi-engine
 * context starts none once its engines are warm (one host
 * thread per GPU, persistent). */
uint64_t mbft_debug_threads_started(void);
/* Test hook (new): the host end of a resident-kernel verify -- nparts (1..16)
 * partial comb sums in the device's limb format (40 words each: X, Y, ZZ, ZZZ
 * as 9 29-bit Montgomery limbs, then a flags word, 1 = infinity) joined and
 * x-checked against r (32 B big-endian).  0 accept, 1 reject. */
int mbft_debug_host_join(const uint32_t* part, int nparts, const uint8_t* r_be);
/* Test hook (new): a resident call's scalars as the host computes them for the
 * kernel (SrvSlot::u) -- u1 = e s^-1, u2 = r s^-1 mod N, 8 little-endian words
 * each, from e, r, s (32 B big-endian each); zeros when s is 0 or >= N.
 * crypto/ecdsa.Verify's u1, u2 (sample/authentication/crypto.go:86). */
int mbft_debug_host_scalars(const uint8_t* e, const uint8_t* r, const uint8_t* s, uint32_t u[16]);
/* Concurrent batches on one GPU (new; the reference calls the authenticator
 * from every peer's and client's stream goroutine at once, api/api.go:132).
 * With lanes > 1, up to `lanes` calls of mbft_verify_batch{,_flat},
 * mbft_check_batch{,_flat} and mbft_verify_message_authen_tag run at the
 * same time: each leases a lane (its own staging, device scratch, streams,
 * s^-1 pipeline and host workers) and shares the context's tables and key
 * store, so their copies and kernels overlap on the device.  The USIG epoch
 * step of a verify batch is applied under the context's lock, one batch at
 * a time, each batch in its own call order -- the outcome of some sequential
 * order of the concurrent calls, as under the reference's scheme lock
 * (crypto.go:198-199).  Key, role and window changes wait for the batches in
 * flight.  Every other entry point keeps running one at a time.  lanes = 1
 * (default) serialises every call on the context.  1 <= lanes <= 64. */
int mbft_set_concurrency(mbft_ctx* ctx, int lanes);
int mbft_get_concurrency(const mbft_ctx* ctx);
/* Comb windows planned from the device's free HBM and the key counts per
 * role (new; what the Go binding uses when no window is configured):
 * greedy over the upgrades with the most table additions saved per verify
 * per byte (a key class weighted by its share of a replica's verifies:
 * ~n USIG UIs and one client signature per request), leaving 6 GiB for
 * batch scratch.  One static signer gets 29 / 29; 33 USIG keys and a
 * client get a generator and key windows that fit together. */
int mbft_plan_windows(int device, size_t n_replica, size_t n_usig, size_t n_client, int* g_wbits,
                      int* replica_wbits, int* usig_wbits, int* client_wbits);
/* mbft_verify_batch over flat buffers: call i = (roles[i], ids[i],
 * msgs[msg_off[i] .. msg_off[i+1]), tags[tag_off[i] .. tag_off[i+1])).  No
 * pointers inside the arguments, so Go can pass its own slices (cgo forbids
 * Go pointers stored in C memory, which an mbft_item array would need). */
int mbft_verify_batch_flat(mbft_ctx* ctx, const uint32_t* roles, const uint32_t* ids,
                           const uint8_t* msgs, const uint64_t* msg_off, const uint8_t* tags,
                           const uint64_t* tag_off, size_t n, uint8_t* status_out);
/* The compact flat form (new): the same calls with 1-byte roles and 32-bit
 * offsets (a batch's message and tag bytes each below 4 GiB).  With the
 * buffers in library page-locked memory a call crosses PCIe in 13 bytes plus
 * its message and tag instead of 24 plus them.  For the ECDSA roles the
 * verdict depends on the message only through e = (msg || SHA256(""))[0:32]
 * (crypto.go:113-126: Sum(m) appends the empty digest, Verify reads 32
 * bytes), so a caller may pass those 32 bytes as the message -- copied, not
 * hashed -- and the statuses are the same (the Go binding does: 32 B instead
 * of 47 for a REQUEST).  Offsets are checked where they are read: with the
 * device decode each call's fields must lie in the batch's byte ranges in
 * order, else MBFT_ERR_ARG (statuses unspecified, no state changed). */
int mbft_verify_batch_flat32(mbft_ctx* ctx, const uint8_t* roles, const uint32_t* ids,
                             const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* tags,
                             const uint32_t* tag_off, size_t n, uint8_t* status_out);
/* Library-owned page-locked host memory (new).  When EVERY buffer of a
 * mbft_verify_batch_flat / mbft_check_batch_flat call (roles, ids, msg_off,
 * tag_off, and the used ranges of msgs and tags) lies in such allocations,
 * the calls travel to the GPU raw, chunk by chunk, and are decoded there
 * (role / key dispatch, Go-exact DER, the Sum(m) digest, the USIG UI / cert
 * split and digest chain; kernels.hip k_prepare): the host reads none of
 * their bytes except the roles (a scan for USIG calls, whose epoch step
 * stays on the host in call order).  Results are identical to the host
 * decode.  A status_out in such memory also receives the statuses straight
 * from the GPU.  The Go binding marshals its batches into these buffers
 * (cgo: C memory).  mbft_host_alloc: MBFT_ERR_NOMEM on failure;
 * mbft_host_free: MBFT_ERR_ARG for a pointer it did not return. */
int mbft_host_alloc(size_t bytes, void** out);
int mbft_host_free(void* p);
/* Device decode on (1, default) or off (0: always the host decode). */
int mbft_set_device_prepare(mbft_ctx* ctx, int enabled);
/* Kernel for batches below the batched-s^-1 threshold (new; tuning and
 * tests): up to split_max items take k_verify_split (one item per 4-wave
 * workgroup, the comb windows split over the waves: the lowest latency for
 * single calls, s^-1 per wave), larger ones the lane-pair / lane-quad
 * kernels (mbft_set_small_batch_inverse).
 * split_max < 0: env MBFT_SPLIT_MAX, default 256; 0: pairs only. */
int mbft_set_small_batch_form(mbft_ctx* ctx, long split_max);
/* The form of the small batches past the split kernel's (new; tuning and
 * tests): 2 k_verify_quads (an item per lane quad, each lane half of one
 * scalar's windows) with s^-1 by each wave inside it (one wave-cooperative
 * inversion per 16 items); 3 the batched per-wave s^-1 into planes first
 * (k_ninv_local), then k_verify_quads; 1 the planes, then k_verify_pairs (an
 * item per lane pair); 0 k_verify_pairs inverting s per lane (divsteps); -1
 * env MBFT_PAIRS_PLANES / MBFT_QUADS / MBFT_QUADS_INLINE (default 2).
 * MBFT_ERR_ARG outside -1..3. */
int mbft_set_small_batch_inverse(mbft_ctx* ctx, int mode);
/* Two-phase form of the same semantics, for callers that must keep their
 * own per-call order (the core's stream loops):
 *   mbft_check_batch   the pure part of n calls, all signatures on the GPU
 *                      at once, NO state touched: pure_out[i] = the status
 *                      call i gets if its USIG epoch check passes;
 *   mbft_resolve_checked  later, per call and in call order: the host part
 *                      of the call again plus the USIG epoch step
 *                      (crypto.go:219-236) over `pure` -- no GPU work.
 * resolve_checked(call, check(call)) == verify_message_authen_tag(call). */
int mbft_check_batch(mbft_ctx* ctx, const mbft_item* items, size_t n, uint8_t* pure_out);
int mbft_check_batch_flat(mbft_ctx* ctx, const uint32_t* roles, const uint32_t* ids,
                          const uint8_t* msgs, const uint64_t* msg_off, const uint8_t* tags,
                          const uint64_t* tag_off, size_t n, uint8_t* pure_out);
int mbft_check_batch_flat32(mbft_ctx* ctx, const uint8_t* roles, const uint32_t* ids,
                            const uint8_t* msgs, const uint32_t* msg_off, const uint8_t* tags,
                            const uint32_t* tag_off, size_t n, uint8_t* pure_out);
int mbft_resolve_checked(mbft_ctx* ctx, uint32_t role, uint32_t id, const uint8_t* msg,
                         size_t msg_len, const uint8_t* tag, size_t tag_len, uint8_t pure);
int mbft_generate_message_authen_tag(mbft_ctx* ctx, uint32_t role, const uint8_t* msg,
                                     size_t msg_len, uint8_t* tag_out, size_t tag_cap,
                                     size_t* tag_len);

/* crypto/ecdsa.Verify core over decoded items.  e, r, s: n x 32 bytes
 * big-endian (e = hashToInt input, i.e. the left-most 32 bytes of the
 * digest, zero-padded on the LEFT if the digest is shorter); slots from
 * mbft_key_slot / mbft_register_points.  status: n bytes (mbft_status). */
int mbft_verify_prehashed(mbft_ctx* ctx, const uint8_t* e, const uint8_t* r, const uint8_t* s,
                          const uint32_t* slots, size_t n, uint8_t* status);
int mbft_verify_prehashed_device(mbft_ctx* ctx, const uint8_t* d_e, const uint8_t* d_r,
                                 const uint8_t* d_s, const uint32_t* d_slots, size_t n,
                                 uint8_t* d_status, void* hip_stream);

/* Bulk ECDSA signing over decoded digests, for synthetic load generation
 * and tests (the signature format of crypto.go:63-76).  priv32: nkeys x 32 B
 * big-endian scalars; key_idx: n indices (NULL = key 0); e: n x 32 B; r, s:
 * n x 32 B big-endian outputs.  Deterministic nonce.  NOT CONSTANT-TIME:
 * its memory accesses depend on the nonce; never give it a key that
 * protects anything. */
int mbft_sign_prehashed(mbft_ctx* ctx, const uint8_t* priv32, size_t nkeys,
                        const uint32_t* key_idx, const uint8_t* e, size_t n, uint8_t* r_out,
                        uint8_t* s_out);
int mbft_sign_prehashed_device(mbft_ctx* ctx, const uint8_t* d_priv32, const uint32_t* d_key_idx,
                               const uint8_t* d_e, size_t n, uint8_t* d_r, uint8_t* d_s,
                               void* hip_stream);

/* Signing with GIVEN nonces k (n x 32 B big-endian, 1 <= k < N): r = x(kG)
 * mod N, s = k^-1 (e + r d) mod N; a bad nonce gives r = s = 0.  For
 * constructing crafted inputs (bench.py's adversarial lines: items whose u2
 * has a zero comb window), never used for real tags. */
int mbft_sign_nonce_device(mbft_ctx* ctx, const uint8_t* d_priv32, const uint32_t* d_key_idx,
                           const uint8_t* d_e, const uint8_t* d_k, size_t n, uint8_t* d_r,
                           uint8_t* d_s, void* hip_stream);

/* SHA-256 stage on the GPU over device buffers, on the caller's stream
 * (north_star item 3: AuthenBytes construction feeds a GPU SHA-256 stage).
 *   mbft_request_digests_device: the ECDSA-role digest input of n REQUESTs,
 *     e_i = (AuthenBytes(REQUEST_i) || SHA256(""))[0:32]
 *         = "REQUEST" || seq_be64 || SHA256(op_i)[0:17]
 *     (messages/authen.go:33,54-56 + sample/authentication/crypto.go:121);
 *     ops: n x op_len bytes back to back; seq: n u64.
 *   mbft_sha256_device: out_i = SHA256(data[off_i, off_{i+1})), the hashsum
 *     of messages/authen.go:78-82; off: n + 1 byte offsets.
 *   mbft_usig_digests_device: e_i = SHA256(SHA256(m_i) || epoch_le64 ||
 *     counter_le64), the USIG signed digest (usig/sgx/sgx-usig.go:99-101,
 *     usig/sgx/usig-enclave.go:204-214); m_i = data[off_i, off_{i+1}).
 * Outputs are n x 32 bytes (big-endian digest bytes). */
int mbft_request_digests_device(mbft_ctx* ctx, const uint64_t* d_seq, const uint8_t* d_ops,
                                uint32_t op_len, size_t n, uint8_t* d_e, void* hip_stream);
int mbft_sha256_device(mbft_ctx* ctx, const uint8_t* d_data, const uint64_t* d_off, size_t n,
                       uint8_t* d_out, void* hip_stream);
int mbft_usig_digests_device(mbft_ctx* ctx, const uint8_t* d_data, const uint64_t* d_off,
                             const uint64_t* d_epoch, const uint64_t* d_counter, size_t n,
                             uint8_t* d_e, void* hip_stream);

/* Kernel timing: when enabled, HIP events bracket the batched-inversion and
 * verify kernels of every verify call, on the stream they run on.
 * mbft_profile_read fills out[0] = total verify-kernel ms, out[1] = total
 * inversion ms, out[2] = batches, out[3] = items, and resets the totals. */
int mbft_profile_enable(mbft_ctx* ctx, int enable);
int mbft_profile_read(mbft_ctx* ctx, double out[4]);
/* Host-side stage times of mbft_verify_batch since the last read (always
 * collected): out[0] = batches, out[1] = items, out[2] = host per-call work
 * (role/key lookup, DER decode, digest construction, staging writes; ms,
 * overlapped with the previous chunk's transfers and kernels), out[3] = wait
 * for the GPU after the last chunk was enqueued (ms), out[4] = in-order
 * resolution incl. the USIG epoch replay (ms), out[5] = wall total (ms).
 * Resets the totals. */
int mbft_profile_stages(mbft_ctx* ctx, double out[6]);
/* The device message layer (mbft_validate_messages_flat,
 * mbft_check_messages_flat) while profiling is enabled, from HIP events:
 * out[0] = calls, out[1] = H2D ms (the records' and arena's uploads on the
 * copy stream, first copy start to last copy end), out[2] = device ms (first
 * copy start to the end of the last kernel / download), out[3] = bytes
 * uploaded; summed over the context and its lanes, then reset. */
int mbft_profile_msg_layer(mbft_ctx* ctx, double out[4]);

/* ---------------------------------------------------------------------------
 * MinBFT message layer.
 *
 * mbft_message flattens a message's authenticated fields
 * (messages/authen.go:52-76, messages/api.go):
 *   REQUEST          client_id, seq, op, sig
 *   REPLY            replica_id, client_id, seq, op (= result), sig
 *                    (client side only: mbft_validate_replies)
 *   PREPARE          replica_id (primary), view, client_id, seq, op, sig (of
 *                    the embedded REQUEST), ui_counter/ui_cert
 *   COMMIT           replica_id, prep_replica_id, view, client_id, seq, op,
 *                    sig, prep_ui_counter/prep_ui_cert (the embedded
 *                    PREPARE's UI), ui_counter/ui_cert
 *   REQ-VIEW-CHANGE  view (= the new view)
 * `stream` identifies the peer/client stream the message arrived on. */
enum mbft_msg_type {
  MBFT_MSG_REQUEST = 1,
  MBFT_MSG_REPLY = 2,
  MBFT_MSG_PREPARE = 3,
  MBFT_MSG_COMMIT = 4,
  MBFT_MSG_REQ_VIEW_CHANGE = 5
};

typedef struct mbft_message {
  uint32_t type;
  uint32_t stream;
  uint32_t replica_id;
  uint32_t prep_replica_id;
  uint64_t view;
  uint32_t client_id;
  uint32_t reserved;
  uint64_t seq;
  const uint8_t* op;
  size_t op_len;
  const uint8_t* sig;
  size_t sig_len;
  uint64_t ui_counter;
  const uint8_t* ui_cert;
  size_t ui_cert_len;
  uint64_t prep_ui_counter;
  const uint8_t* prep_ui_cert;
  size_t prep_ui_cert_len;
} mbft_message;

/* Validation result per message: 0 = valid, else (stage << 8) | mbft_status
 * of the failing check (status 0 for checks that are not authenticator
 * calls). */
enum mbft_stage {
  MBFT_ST_REQUEST_SIG = 1,         /* core/request.go:146-150 (also inside PREPARE/COMMIT) */
  MBFT_ST_NOT_PRIMARY = 2,         /* core/prepare.go:51-53 "Prepare from backup" */
  MBFT_ST_PREPARE_UI = 3,          /* core/prepare.go:59-61 + core/usig-ui.go:62-77 */
  MBFT_ST_COMMIT_FROM_PRIMARY = 4, /* core/commit.go:78-80 */
  MBFT_ST_COMMIT_UI = 5,           /* core/commit.go:86-88 */
  MBFT_ST_NOT_IMPLEMENTED = 6,     /* core/message-handling.go:418-419 (ReqViewChange) */
  MBFT_ST_STREAM_STOPPED = 7,      /* an earlier message of the stream was rejected
                                      (core/message-handling.go:217-220) */
  MBFT_ST_REPLY_SIG = 8,           /* client/message-handling.go:161-170 */
  MBFT_ST_AFTER_PANIC = 9,         /* an earlier message made Go panic (crypto.go:82-84) */
  MBFT_ST_UNKNOWN_TYPE = 10,       /* a REPLY in a replica's stream: the message
                                      validator panics (core/message-handling.go:420-421) */
  MBFT_ST_REPLY_CLIENT_ID = 11     /* client/message-handling.go:163-165 "Client ID mismatch" */
};

enum mbft_validate_flags { MBFT_VF_NO_STREAM_STOP = 1, MBFT_VF_NO_PANIC_STOP = 2 };

/* messages.AuthenBytes (messages/authen.go:27-50): writes into out (cap
 * bytes), *len = required size (MBFT_ERR_ARG if cap is too small). */
int mbft_authen_bytes(const mbft_message* m, uint8_t* out, size_t cap, size_t* len);

/* The digest input e of the authenticator call over AuthenBytes(msgs[i]),
 * built on the GPU from the raw fields (SHA256(op) by k_sha256_var, the
 * AuthenBytes layout of messages/authen.go:52-76 in registers by
 * k_authen_e), one host round trip:
 *   kind 0  REQUEST, ECDSA role:  e = (AuthenBytes || SHA256(""))[0:32]
 *   kind 1  REPLY, ECDSA role:    the same over the REPLY layout
 *   kind 2  PREPARE, USIG:  e = SHA256(SHA256(AuthenBytes) || epochs[i]_le || counters[i]_le)
 *   kind 3  COMMIT, USIG:   the same over the COMMIT layout (prep_replica_id,
 *                           prep_ui_counter)
 * (crypto.go:121; sgx-usig.go:99-101, usig-enclave.go:204-214).  e_out: n x
 * 32 bytes.  mbft_validate_messages / _replies use the same stage. */
int mbft_authen_digests(mbft_ctx* ctx, const mbft_message* msgs, size_t n, uint32_t kind,
                        const uint64_t* epochs, const uint64_t* counters, uint8_t* e_out);

/* Validates n messages in order exactly as the core's messageValidator would,
 * one stream loop per `stream` value, with all signature checks of the batch
 * on the GPU (identical authenticator calls verified once).  n_replicas is
 * the `n` of isPrimary (view mod n).  out: n results as above. */
int mbft_validate_messages(mbft_ctx* ctx, const mbft_message* msgs, size_t n, uint32_t n_replicas,
                           uint32_t flags, int32_t* out);

/* The same validation over a FLAT batch (new; replaces the same
 * core/message-handling.go:409-424 validator loop as mbft_validate_messages):
 * one fixed-size record per message with the variable-length fields as
 * offsets into one byte arena -- no pointers, so Go can marshal a batch
 * straight into C memory.  When `recs` and `bytes` lie in library page-locked
 * memory (mbft_host_alloc), the whole message layer runs on the GPU: the
 * records and bytes go up raw, and the candidate calls of every message, their
 * content hashes and the deduplication (a device hash table, first occurrence
 * in message order wins, every hash hit compared in full), the AuthenBytes +
 * SHA-256 digests, Go-exact DER, the USIG UI / cert split and the key lookups
 * are all kernels (msg_kernels.hip); the host only replays the results in
 * message order (stream stop, panic stop, USIG epoch state).  Otherwise (or
 * past 2^28 messages in one call) the records are turned into mbft_message
 * structs over `bytes` and validated by mbft_validate_messages.  Results are identical either way.  Offsets are
 * byte offsets into `bytes` (nbytes long); a field of length 0 may carry any
 * offset.  mbft_pack_messages builds such a batch from mbft_message structs
 * (the bytes each message points to, copied): *used = the arena bytes the
 * batch needs (recs == NULL: only that), MBFT_ERR_ARG when cap is too small. */
typedef struct mbft_msg_rec {
  uint32_t type;
  uint32_t stream;
  uint32_t replica_id;
  uint32_t prep_replica_id;
  uint32_t client_id;
  uint32_t op_len;
  uint32_t sig_len;
  uint32_t ui_cert_len;
  uint32_t prep_ui_cert_len;
  uint32_t reserved;
  uint64_t view;
  uint64_t seq;
  uint64_t ui_counter;
  uint64_t prep_ui_counter;
  uint64_t op_off;
  uint64_t sig_off;
  uint64_t ui_cert_off;
  uint64_t prep_ui_cert_off;
} mbft_msg_rec;

int mbft_validate_messages_flat(mbft_ctx* ctx, const mbft_msg_rec* recs, size_t n,
                                const uint8_t* bytes, size_t nbytes, uint32_t n_replicas,
                                uint32_t flags, int32_t* out);
int mbft_pack_messages(const mbft_message* msgs, size_t n, mbft_msg_rec* recs, uint8_t* bytes,
                       size_t cap, size_t* used);

/* The same validation split in two, like mbft_check_batch /
 * mbft_resolve_checked (new; for the core's stream loop,
 * core/message-handling.go:204-246, which validates each message right
 * before processing it and ends the stream at the first error):
 *   mbft_check_messages_flat  every signature, digest, DER / UI decode and key
 *                      lookup of the batch on the GPU at once (the device
 *                      message layer above), NO state read or written; the
 *                      per-message checks are kept in *out;
 *   mbft_resolve_message  later, per message, in the caller's order: message
 *                      i's result (0, or (stage << 8) | status, as above),
 *                      applying the USIG epoch step (crypto.go:219-236) to
 *                      the context's state at that moment -- no GPU work.
 * No stream stop and no panic stop: each message's own result (the caller's
 * loop stops itself; MBFT_MALFORMED_DER at MBFT_ST_REQUEST_SIG /
 * MBFT_ST_REPLY_SIG and MBFT_ST_UNKNOWN_TYPE are where Go panics).
 * Resolving messages 0 .. n-1 in order gives what mbft_validate_messages_flat
 * gives with MBFT_VF_NO_STREAM_STOP | MBFT_VF_NO_PANIC_STOP; a message never
 * resolved leaves the epoch state untouched, as a message the reference never
 * validates.  recs / bytes outside library page-locked memory are staged into
 * the engine's own first.  Runs on a concurrency lane (mbft_set_concurrency)
 * when there are several; resolve takes the context lock briefly.
 * mbft_msg_batch_free releases the batch (any time after the check). */
typedef struct mbft_msg_batch mbft_msg_batch;
int mbft_check_messages_flat(mbft_ctx* ctx, const mbft_msg_rec* recs, size_t n, const uint8_t* bytes,
                             size_t nbytes, uint32_t n_replicas, mbft_msg_batch** out);
int mbft_resolve_message(mbft_ctx* ctx, mbft_msg_batch* batch, size_t i);
/* count consecutive messages i0 .. i0+count-1 resolved in order into out[]:
 * the same as count mbft_resolve_message calls, one lock and one call. */
int mbft_resolve_messages(mbft_ctx* ctx, mbft_msg_batch* batch, size_t i0, size_t count,
                          int32_t* out);
void mbft_msg_batch_free(mbft_msg_batch* batch);
/* Coalescing of concurrent mbft_check_messages_flat calls (new; the core
 * runs one stream loop per peer connection, core/message-handling.go:
 * 250-275, so a replica's streams check their batches at the same time).
 * When enabled, a call that arrives while another pass holds the engine
 * queues; the first queued caller leads the next pass, which takes every
 * queued batch with the same n_replicas (up to max_messages messages; 0:
 * 2^20) and checks them as ONE device pass -- records and arenas
 * concatenated into the library's page-locked staging, identical calls
 * across the batches verified once -- and every caller gets its own
 * mbft_msg_batch (results exactly as if checked alone: a check touches no
 * state; the USIG epoch step stays in each caller's resolve).  A caller
 * whose records would fail alone (unknown type, field outside its arena)
 * gets MBFT_ERR_ARG and the others are unaffected.  max_wait_us > 0 lets a
 * leader wait that long for company first.  Default: disabled.
 * mbft_check_coalescing_stats: out[0] passes, out[1] caller batches,
 * out[2] messages since the last call (then reset). */
int mbft_set_check_coalescing(mbft_ctx* ctx, int enabled, uint32_t max_wait_us, size_t max_messages);
int mbft_check_coalescing_stats(mbft_ctx* ctx, double out[3]);
/* Small checks (new): a check pass of at most max_messages messages (one
 * caller's batch, or a coalesced pass; default 512, 0 = never) skips the
 * device message layer's fixed cost -- record upload, dedup table, scan,
 * several launches, two host waits -- for the latency of the core's
 * one-message-at-a-time streams (a client's REQUEST stream is strictly
 * sequential, core/message-handling.go:399): the checks and candidate calls
 * are built and deduplicated on the host (content hash, full compares), the
 * AuthenBytes digests hashed on the host (SHA extensions), and the unique
 * calls verified in ONE launch of the small-batch kernel (from zero-copy
 * staging up to 256 calls, s^-1 inverted on the host up to 64) -- the
 * lone-call path.  1 message: ~36 us against ~270 us through the device
 * layer (15-23 us through the resident verifier); 256 messages ~165 us
 * against ~430 us, 512 messages ~315 us against ~440-500 us, 1024 ~500 us
 * against ~450-480 us (tools/lowload_probe.py), hence 512.  Identical
 * results; records
 * and arena may lie in any host memory. */
int mbft_set_small_check(mbft_ctx* ctx, size_t max_messages);

/* Client side: validates n REPLY messages as the client `client_id` does
 * (client/message-handling.go:93-110,140-170): ClientID mismatch ->
 * MBFT_ST_REPLY_CLIENT_ID, else VerifyMessageAuthenTag(ReplicaAuthen,
 * replica_id, AuthenBytes(REPLY), sig) -> 0 or (MBFT_ST_REPLY_SIG << 8 |
 * status).  A rejected REPLY does not stop its stream (the client only logs
 * it); a malformed DER signature panics (then MBFT_ST_AFTER_PANIC, unless
 * MBFT_VF_NO_PANIC_STOP).  Non-REPLY messages -> MBFT_ERR_ARG. */
int mbft_validate_replies(mbft_ctx* ctx, const mbft_message* msgs, size_t n, uint32_t client_id,
                          uint32_t flags, int32_t* out);
/* The same over a flat batch (records + one byte arena, as
 * mbft_validate_messages_flat; new): what the Go client's batched reply loop
 * marshals (go/gpuauth/replies.go).  Batches of up to mbft_set_small_check's
 * size take the small route (AuthenBytes hashed on the host, one zero-copy
 * verify launch), larger ones the GPU digest stage. */
int mbft_validate_replies_flat(mbft_ctx* ctx, const mbft_msg_rec* recs, size_t n, const uint8_t* bytes,
                               size_t nbytes, uint32_t client_id, uint32_t flags, int32_t* out);

/* Host-only helpers (no GPU). */
/* encoding/asn1 DER decode of struct{R, S *big.Int}.
 * Returns 1 on success, 0 on a Go asn1 error.  On success: *consumed = bytes
 * of the outer SEQUENCE (the rest is Go's `rest`); r32/s32 receive the value
 * if 0 < value < 2^256, else zero (Go: r <= 0 or r >= N -> Verify false). */
int mbft_der_parse_sig(const uint8_t* sig, size_t len, uint8_t r32[32], uint8_t s32[32],
                       size_t* consumed);
void mbft_sha256(const uint8_t* data, size_t len, uint8_t out[32]);
/* mbft_sha256 through one host compression (test hook): form 0 the portable
 * one, form 1 the x86 SHA extensions (MBFT_ERR_STATE when the CPU lacks
 * them).  mbft_sha256 and every host digest use form 1 where available. */
int mbft_debug_sha256(int form, const uint8_t* data, size_t len, uint8_t out[32]);

#ifdef __cplusplus
}
#endif

#endif /* MINBFT_GPU_H */
