// Package gpuauth is a drop-in api.Authenticator for MinBFT backed by the
// MI355X batch authenticator (include/minbft_gpu.h, minbft_amd/libminbft_amd.so).
//
// It keeps the reference contract bit for bit (api/api.go:133-144,
// sample/authentication/authenticator.go:121-141): VerifyMessageAuthenTag
// returns nil exactly when the reference does, an error otherwise, and
// panics where EcdsaSigCipher.Verify panics (malformed DER in an ECDSA role,
// sample/authentication/crypto.go:82-84).  On top of it:
//
//   - VerifyBatch: n calls verified together on the GPU, results identical to
//     calling VerifyMessageAuthenTag on them in order (USIG epoch capture,
//     crypto.go:219-236, replayed in call order by the library);
//   - CheckMessages (api.MessageBatchChecker, messages.go): a batch of
//     received messages as raw fields; AuthenBytes, SHA-256, DER / UI
//     decode and every signature on the GPU in one round trip
//     (mbft_check_messages_flat), no state touched; each message is then
//     validated in the core's own order (mbft_resolve_message, the USIG
//     epoch step included).  This is what the batched core stream loop
//     (../core/message-handling-batch.go) uses: the core keeps its
//     per-message, per-stream order and its code, and hashes nothing.
//
// Generation never touches the GPU: GenerateMessageAuthenTag signs on the
// CPU with the reference's own scheme (PublicAuthenScheme{crypto.SHA256,
// EcdsaSigCipher}, crypto.go:63-76,113-116: Go's constant-time P-256), or
// delegates to Config.Generator (the reference authenticator, which also
// owns the SGX USIG).  The library's bulk signer (k_sign) is for synthetic
// load only.
//
// Concurrency: any number of goroutines may call every method at once.
// Batches are marshalled into a pool of arenas (one per in-flight batch), and
// the library runs up to Config.Concurrency check batches at the same time
// on one GPU (mbft_set_concurrency: independent scratch and streams per
// batch, shared key tables); the USIG epoch step is serialised in the
// library, batch by batch, as the reference's scheme lock serialises calls.
//
// cgo pointer rules: batches are marshalled into library-owned page-locked
// C memory (mbft_host_alloc; the GPU then decodes them); single calls pass
// Go memory only as direct arguments (mbft_verify_message_authen_tag,
// mbft_resolve_checked), never stored in C memory, so the package is clean
// under GODEBUG=cgocheck=2.
//
// Go 1.11 compatible (the reference's go.mod:30 and CI matrix 1.11 / 1.14):
// no unsafe.Slice, no big.Int.FillBytes, no %w, no signed shift counts;
// tests/test_go_compat.py checks it.  This package is written against the
// C-ABI and is not built in this repository's image (no Go toolchain); see
// INTEGRATION.md.
package gpuauth

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../minbft_amd -lminbft_amd -Wl,-rpath,${SRCDIR}/../../minbft_amd
#include <stdlib.h>
#include "minbft_gpu.h"
*/
import "C"

import (
	"crypto"
	"crypto/ecdsa"
	"crypto/elliptic"
	"fmt"
	"math/big"
	"unsafe"

	"github.com/hyperledger-labs/minbft/api"
	authen "github.com/hyperledger-labs/minbft/sample/authentication"
)

// Config selects the devices and the comb-table windows (include/minbft_gpu.h:
// HBM cost per window).  Zero values take the defaults below.
type Config struct {
	// Devices: the first builds the context, every other one gets an engine
	// with replicas of all tables; host batches are sharded across them
	// (no collective).  Default {0}.
	Devices []int
	// Windows in bits (4..29).  Zero: sized from the HBM budget by
	// DefaultWindows (include/minbft_gpu.h, mbft_plan_windows).
	GeneratorWindow, ReplicaWindow, USIGWindow, ClientWindow int
	// Private keys of the ECDSA roles this node signs as (CPU signing with
	// the reference scheme, crypto.go:63-76), used when Generator is nil.
	PrivateKeys map[api.AuthenticationRole]*ecdsa.PrivateKey
	// Generator, if set, generates every tag: the reference authenticator
	// built by authen.New / authen.NewWithSGXUSIG (USIG UIs stay in the SGX
	// enclave).  USIGGenerator is the older name for the USIG role only.
	Generator     api.Authenticator
	USIGGenerator api.Authenticator
	// Concurrency: check batches the library runs at the same time on one
	// GPU (mbft_set_concurrency, default 4); 1 serialises them.
	Concurrency int
	// Coalesce verifies concurrent VerifyMessageAuthenTag calls (goroutines)
	// together: calls arriving while a batch is on the GPU share the next
	// one (mbft_set_coalescing).  CoalesceWaitMicros > 0 also lets a lone
	// call wait that long for company; CoalesceMaxBatch caps a batch.
	Coalesce           bool
	CoalesceWaitMicros uint32
	CoalesceMaxBatch   uint32
	// ResidentSlots: VerifyMessageAuthenTag calls go to a verify kernel kept
	// on the GPU (mbft_set_resident), one mailbox slot per concurrent call,
	// no kernel launch per call; calls past the slots take the coalescer.
	// Default 32 (a replica's peer and client goroutines calling at once);
	// negative turns it off.
	ResidentSlots int
	// SeparateChecks turns off the merging of concurrent CheckMessages
	// calls (on by default: the core's stream loops -- one goroutine per
	// connection -- check their batches at the same time, and the library
	// runs the batches queued behind a pass as ONE device pass, identical
	// calls across streams verified once; mbft_set_check_coalescing).
	// Every caller still gets exactly its own batch's results.
	SeparateChecks bool
	// KeyStore, if set, is consulted for any (role, id) the context does
	// not hold when a call by it arrives: the reference verifies every id
	// its key store has (keymanager.go:96-101), so that key is registered
	// (at its role's window) before the call's batch runs (keys.go).
	KeyStore PublicKeyStore
}

// Authenticator implements api.Authenticator and api.MessageBatchChecker on
// the GPU.
type Authenticator struct {
	ctx     *C.mbft_ctx
	gen     api.Authenticator
	usigGen api.Authenticator
	priv    map[api.AuthenticationRole]*ecdsa.PrivateKey

	arenas arenaPool   // batches are marshalled here (library page-locked memory)
	keys   keyRegistry // the (role, id) pairs the context holds (keys.go)
}

var _ api.Authenticator = (*Authenticator)(nil)
var _ api.MessageBatchChecker = (*Authenticator)(nil)

// Call is one VerifyMessageAuthenTag call (api.AuthenCall).
type Call = api.AuthenCall

// ecdsaScheme is the reference's scheme for the ECDSA roles
// (authenticator.go:100-101), used for signing on the CPU.
var ecdsaScheme = &authen.PublicAuthenScheme{HashScheme: crypto.SHA256, SigCipher: &authen.EcdsaSigCipher{}}

// New builds the authenticator over the public keys of every role
// (as loaded by LoadSimpleKeyStore, keymanager.go:179-227).
func New(keys map[api.AuthenticationRole]map[uint32]*ecdsa.PublicKey, usigEnabled bool,
	cfg Config) (*Authenticator, error) {
	devices := cfg.Devices
	if len(devices) == 0 {
		devices = []int{0}
	}
	var ctx *C.mbft_ctx
	if rc := C.mbft_ctx_create(C.int(devices[0]), &ctx); rc != C.MBFT_OK {
		return nil, fmt.Errorf("mbft_ctx_create(%d): %d", devices[0], int(rc))
	}
	a := &Authenticator{ctx: ctx, gen: cfg.Generator, usigGen: cfg.USIGGenerator,
		priv: cfg.PrivateKeys}
	a.arenas.init(16)
	fail := func(what string, rc C.int) (*Authenticator, error) {
		err := fmt.Errorf("%s: %d (%s)", what, int(rc), C.GoString(C.mbft_last_error(ctx)))
		a.Close()
		return nil, err
	}
	nkeys := map[api.AuthenticationRole]int{}
	for role, m := range keys {
		nkeys[role] = len(m)
	}
	w := DefaultWindows(nkeys, cfg)
	a.keys.init(cfg.KeyStore, w)
	if rc := C.mbft_set_generator_window(ctx, C.int(w.Generator)); rc != C.MBFT_OK {
		return fail("mbft_set_generator_window", rc)
	}
	for _, d := range devices[1:] {
		if rc := C.mbft_ctx_add_device(ctx, C.int(d)); rc != C.MBFT_OK {
			return fail(fmt.Sprintf("mbft_ctx_add_device(%d)", d), rc)
		}
	}
	for role, m := range keys {
		if roleByte(role) == 0 {
			continue // no scheme for the role (authenticator.go:126-129): its calls are rejected anyway
		}
		kw := w.Replica
		switch role {
		case api.ClientAuthen:
			kw = w.Client
		case api.USIGAuthen:
			kw = w.USIG
		}
		if rc := C.mbft_set_key_window(ctx, C.int(kw)); rc != C.MBFT_OK {
			return fail("mbft_set_key_window", rc)
		}
		C.mbft_add_role(ctx, C.uint32_t(role))
		for id, pk := range m {
			xy, err := rawXY(pk)
			if err != nil {
				a.Close()
				return nil, err
			}
			if rc := C.mbft_set_public_key_xy(ctx, C.uint32_t(role), C.uint32_t(id),
				(*C.uint8_t)(unsafe.Pointer(&xy[0]))); rc != C.MBFT_OK {
				return fail(fmt.Sprintf("public key %v/%d", role, id), rc)
			}
			a.keys.add(role, id)
		}
	}
	C.mbft_enable_usig(ctx, cBool(usigEnabled))
	conc := cfg.Concurrency
	if conc == 0 {
		conc = 4
	}
	if rc := C.mbft_set_concurrency(ctx, C.int(conc)); rc != C.MBFT_OK {
		return fail("mbft_set_concurrency", rc)
	}
	if !cfg.SeparateChecks {
		if rc := C.mbft_set_check_coalescing(ctx, 1, 0, 0); rc != C.MBFT_OK {
			return fail("mbft_set_check_coalescing", rc)
		}
	}
	if cfg.Coalesce {
		if rc := C.mbft_set_coalescing(ctx, 1, C.uint32_t(cfg.CoalesceWaitMicros),
			C.uint32_t(cfg.CoalesceMaxBatch)); rc != C.MBFT_OK {
			return fail("mbft_set_coalescing", rc)
		}
	}
	slots := cfg.ResidentSlots
	if slots == 0 {
		slots = 32
	}
	if slots > 0 {
		if rc := C.mbft_set_resident(ctx, C.int(slots)); rc != C.MBFT_OK {
			return fail("mbft_set_resident", rc)
		}
	}
	return a, nil
}

// PublicKeyStore is the part of the reference's key store the constructor
// reads (authen.SimpleKeyStore, keymanager.go:96-101).
type PublicKeyStore interface {
	NodePublicKey(role api.AuthenticationRole, id uint32) (interface{}, error)
}

// KeysFromStore collects the public keys of the given ids per role from a
// key store loaded by authen.LoadSimpleKeyStore (the same keys.yaml the
// reference reads; KeyIDsFromFile lists all its ids).  A role whose key set
// the store has is declared even with no ids (an unknown id is then "invalid
// signature", as in the reference); a role without a key set stays unknown
// ("key set not found"), an id without a key is left out: the GPU
// authenticator then rejects it exactly as the reference does.
func KeysFromStore(ks PublicKeyStore, ids map[api.AuthenticationRole][]uint32) (
	map[api.AuthenticationRole]map[uint32]*ecdsa.PublicKey, error) {
	keys := make(map[api.AuthenticationRole]map[uint32]*ecdsa.PublicKey)
	for role, idl := range ids {
		probe := uint32(0)
		if len(idl) > 0 {
			probe = idl[0]
		}
		if _, err := ks.NodePublicKey(role, probe); err != nil {
			continue // no key set for the role: the role stays unknown
		}
		keys[role] = make(map[uint32]*ecdsa.PublicKey)
		for _, id := range idl {
			pk, err := ks.NodePublicKey(role, id)
			if err != nil || pk == nil {
				continue
			}
			epk, ok := pk.(*ecdsa.PublicKey)
			if !ok {
				return nil, fmt.Errorf("key %v/%d is not an ECDSA public key", role, id)
			}
			keys[role][id] = epk
		}
	}
	return keys, nil
}

// Windows are the comb windows per key class (bits).
type Windows struct {
	Generator, Replica, USIG, Client int
}

// DefaultWindows sizes the comb tables from the device's HBM and the key
// counts (mbft_plan_windows, include/minbft_gpu.h); explicit Config windows
// win.
func DefaultWindows(nkeys map[api.AuthenticationRole]int, cfg Config) Windows {
	var g, r, u, c C.int
	C.mbft_plan_windows(C.int(firstDevice(cfg)), C.size_t(nkeys[api.ReplicaAuthen]),
		C.size_t(nkeys[api.USIGAuthen]), C.size_t(nkeys[api.ClientAuthen]), &g, &r, &u, &c)
	return Windows{
		Generator: orDefault(cfg.GeneratorWindow, int(g)),
		Replica:   orDefault(cfg.ReplicaWindow, int(r)),
		USIG:      orDefault(cfg.USIGWindow, int(u)),
		Client:    orDefault(cfg.ClientWindow, int(c)),
	}
}

func firstDevice(cfg Config) int {
	if len(cfg.Devices) == 0 {
		return 0
	}
	return cfg.Devices[0]
}

// Close releases the GPU context and its tables.  No call may be in flight.
func (a *Authenticator) Close() {
	a.arenas.close()
	if a.ctx != nil {
		C.mbft_ctx_destroy(a.ctx)
		a.ctx = nil
	}
}

// VerifyMessageAuthenTag implements api.Authenticator: one GPU round trip
// (mbft_verify_message_authen_tag; with Config.Coalesce, concurrent calls
// share batches).
func (a *Authenticator) VerifyMessageAuthenTag(role api.AuthenticationRole, id uint32,
	msg []byte, tag []byte) error {
	a.ensureKey(role, id)
	st := C.mbft_verify_message_authen_tag(a.ctx, C.uint32_t(roleByte(role)), C.uint32_t(id), ptr(msg),
		C.size_t(len(msg)), ptr(tag), C.size_t(len(tag)))
	if st < 0 { // a C-ABI failure (HIP error, out of memory): once more (errors.go)
		st = C.mbft_verify_message_authen_tag(a.ctx, C.uint32_t(roleByte(role)), C.uint32_t(id), ptr(msg),
			C.size_t(len(msg)), ptr(tag), C.size_t(len(tag)))
	}
	return a.statusToErr(role, id, int(st))
}

// roleByte is the role the library sees: the reference's three roles
// (api/api.go:98-115) as themselves, any other value -- however large; the
// role is a Go int -- as 0, which the library rejects as MBFT_UNKNOWN_ROLE,
// the reference's "key set not found" / "Unknown role"
// (keymanager.go:96-101, authenticator.go:121-134).  Narrowing the int to
// 8 or 32 bits instead would alias 257 to ReplicaAuthen.
func roleByte(r api.AuthenticationRole) byte {
	switch r {
	case api.ReplicaAuthen, api.USIGAuthen, api.ClientAuthen:
		return byte(r)
	}
	return 0
}

// VerifyBatch verifies calls on the GPU; the result is exactly that of
// VerifyMessageAuthenTag on each call in order (a nil entry is Go's nil; a
// malformed DER tag in an ECDSA role panics, as the reference does, at the
// position of that call).
func (a *Authenticator) VerifyBatch(calls []Call) []error {
	n := len(calls)
	out := make([]error, n)
	if n == 0 {
		return out
	}
	a.ensureKeys(calls)
	ar := a.arenas.get()
	f, ok := ar.flatten(calls)
	if !ok {
		// the batch's bytes do not fit the compact form's 32-bit offsets:
		// verified as consecutive halves, in order (the USIG epoch step runs in
		// call order within and across them, as one batch would); a single
		// call that large goes through the call-level entry (size_t lengths)
		a.arenas.put(ar)
		if n == 1 {
			out[0] = a.VerifyMessageAuthenTag(calls[0].Role, calls[0].ID, calls[0].Msg, calls[0].Tag)
			return out
		}
		copy(out, a.VerifyBatch(calls[:n/2]))
		copy(out[n/2:], a.VerifyBatch(calls[n/2:]))
		return out
	}
	rc := C.mbft_verify_batch_flat32(a.ctx, u8p(f.roles), u32p(f.ids), ptr(f.msgs), u32p(f.msgOff),
		ptr(f.tags), u32p(f.tagOff), C.size_t(n), ptr(f.status))
	if rc < 0 { // once more (errors.go); a failed batch touched no epoch state
		rc = C.mbft_verify_batch_flat32(a.ctx, u8p(f.roles), u32p(f.ids), ptr(f.msgs), u32p(f.msgOff),
			ptr(f.tags), u32p(f.tagOff), C.size_t(n), ptr(f.status))
	}
	if rc != C.MBFT_OK {
		a.arenas.put(ar)
		err := a.failure("mbft_verify_batch_flat32", int(rc))
		for i := range out {
			out[i] = err
		}
		return out
	}
	st := append([]byte(nil), f.status...)
	a.arenas.put(ar)
	for i := range calls {
		out[i] = a.statusToErr(calls[i].Role, calls[i].ID, int(st[i]))
	}
	return out
}

// GenerateMessageAuthenTag implements api.Authenticator on the CPU: the
// reference authenticator (Config.Generator) if given, else the
// reference's ECDSA scheme with Config.PrivateKeys (Sum(m) digest, DER,
// crypto.go:63-76,113-116); the USIG role needs the SGX-backed reference
// authenticator.
func (a *Authenticator) GenerateMessageAuthenTag(role api.AuthenticationRole,
	msg []byte) ([]byte, error) {
	if a.gen != nil {
		return a.gen.GenerateMessageAuthenTag(role, msg)
	}
	if role == api.USIGAuthen {
		if a.usigGen == nil {
			return nil, fmt.Errorf("no USIG to generate UIs")
		}
		return a.usigGen.GenerateMessageAuthenTag(role, msg)
	}
	var sk interface{} // an untyped nil, as the key store returns for no key
	if k := a.priv[role]; k != nil {
		sk = k
	}
	return ecdsaScheme.GenerateAuthenticationTag(msg, sk)
}

// ---------------------------------------------------------------- helpers

// flat is one batch in the compact flat form (mbft_verify_batch_flat32):
// 1-byte roles, 32-bit offsets, and each ECDSA-role message as its 32-byte
// digest prefix e = (msg || SHA256(""))[0:32] -- the only part of it
// crypto/ecdsa.Verify reads (crypto.go:113-126: Sum(m) appends the empty
// digest), copied, not hashed; USIG messages whole (their SHA-256 is taken
// on the GPU).  13 bytes per call plus message and tag cross PCIe.
type flat struct {
	roles, msgs, tags, status []byte
	ids, msgOff, tagOff       []uint32
}

// sha256Empty is SHA256(""), the digest Sum(m) appends (crypto.go:121).
var sha256Empty = [32]byte{0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4, 0xc8,
	0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b,
	0x78, 0x52, 0xb8, 0x55}

// msgPart is what of a call's message goes to the library.
func msgPart(c *Call) int {
	if c.Role == api.USIGAuthen {
		return len(c.Msg)
	}
	return 32
}

// maxArena bounds one arena (the Go 1.11 array-pointer slice idiom needs a
// constant array length); larger batches use Go slices.
const maxArena = 1 << 34

func bytesAt(p unsafe.Pointer, n int) []byte { return (*[maxArena]byte)(p)[:n:n] }

func u32At(p unsafe.Pointer, n int) []uint32 { return (*[maxArena / 4]uint32)(p)[:n:n] }


func arenaAt(p unsafe.Pointer, off int) unsafe.Pointer {
	return unsafe.Pointer(uintptr(p) + uintptr(off))
}

// arena: library-owned page-locked host memory (mbft_host_alloc) one batch
// is marshalled into.  It is C memory, so passing it is clean under the cgo
// pointer rules, and a batch whose buffers all lie in it travels to the GPU
// raw and is decoded there (DER, digest, key; include/minbft_gpu.h): the
// library's host threads read none of its bytes.  Grown on demand; owned by
// one batch at a time (arenaPool).
type arena struct {
	base unsafe.Pointer
	size int
}

func (ar *arena) release() {
	if ar.base != nil {
		C.mbft_host_free(ar.base)
		ar.base, ar.size = nil, 0
	}
}

func (ar *arena) ensure(bytes int) bool {
	if bytes <= ar.size {
		return true
	}
	if bytes > maxArena {
		return false
	}
	ar.release()
	want := bytes + bytes/4
	if want > maxArena {
		want = maxArena
	}
	var p unsafe.Pointer
	if C.mbft_host_alloc(C.size_t(want), &p) != C.MBFT_OK {
		return false
	}
	ar.base, ar.size = p, want
	return true
}

// arenaPool hands one arena to each in-flight batch, so concurrent
// VerifyBatch / CheckMessages calls marshal and run side by side (the library
// overlaps them, mbft_set_concurrency); at most cap idle arenas are kept.
type arenaPool struct {
	free chan *arena
}

func (p *arenaPool) init(n int) { p.free = make(chan *arena, n) }

func (p *arenaPool) get() *arena {
	select {
	case ar := <-p.free:
		return ar
	default:
		return &arena{}
	}
}

func (p *arenaPool) put(ar *arena) {
	select {
	case p.free <- ar:
	default:
		ar.release()
	}
}

func (p *arenaPool) close() {
	for {
		select {
		case ar := <-p.free:
			ar.release()
		default:
			return
		}
	}
}

// maxFlat32: message or tag bytes one compact batch can address.
const maxFlat32 = 1<<32 - 1

// flatten packs calls into the arena in the compact form (8-byte aligned
// regions: offsets, ids, roles, message bytes, tag bytes, statuses); with no
// arena memory it falls back to pointer-free Go slices (passed as
// arguments, never retained by the library; decoded on the host).  false if
// the batch's bytes do not fit 32-bit offsets.
func (ar *arena) flatten(calls []Call) (flat, bool) {
	n := len(calls)
	var ml, tl int
	for i := range calls {
		ml += msgPart(&calls[i])
		tl += len(calls[i].Tag)
	}
	if ml > maxFlat32 || tl > maxFlat32 {
		return flat{}, false
	}
	al := func(x int) int { return (x + 7) &^ 7 }
	var f flat
	if ar.ensure(2*al(4*(n+1)) + al(4*n) + al(n) + al(ml+1) + al(tl+1) + al(n)) {
		o := 0
		take := func(sz int) unsafe.Pointer {
			p := arenaAt(ar.base, o)
			o += al(sz)
			return p
		}
		f.msgOff = u32At(take(4*(n+1)), n+1)
		f.tagOff = u32At(take(4*(n+1)), n+1)
		f.ids = u32At(take(4*n), n)
		f.roles = bytesAt(take(n), n)
		f.msgs = bytesAt(take(ml+1), ml+1)
		f.tags = bytesAt(take(tl+1), tl+1)
		f.status = bytesAt(take(n), n)
	} else {
		f = flat{roles: make([]byte, n), ids: make([]uint32, n), msgs: make([]byte, ml+1),
			tags: make([]byte, tl+1), status: make([]byte, n),
			msgOff: make([]uint32, n+1), tagOff: make([]uint32, n+1)}
	}
	var mo, to int
	f.msgOff[0], f.tagOff[0] = 0, 0
	for i := range calls {
		c := &calls[i]
		f.roles[i] = roleByte(c.Role)
		f.ids[i] = c.ID
		if c.Role == api.USIGAuthen {
			mo += copy(f.msgs[mo:], c.Msg)
		} else { // e = (msg || SHA256(""))[0:32], by copying
			k := copy(f.msgs[mo:mo+32], c.Msg)
			copy(f.msgs[mo+k:mo+32], sha256Empty[:])
			mo += 32
		}
		to += copy(f.tags[to:], c.Tag)
		f.msgOff[i+1] = uint32(mo)
		f.tagOff[i+1] = uint32(to)
	}
	return f, true
}

// put32 writes v (< 2^256) big-endian, left-padded, into dst[0:32] (the
// pre-Go-1.15 form of big.Int.FillBytes).
func put32(dst []byte, v *big.Int) bool {
	b := v.Bytes()
	if len(b) > 32 {
		return false
	}
	for i := 0; i < 32-len(b); i++ {
		dst[i] = 0
	}
	copy(dst[32-len(b):32], b)
	return true
}

func rawXY(pk *ecdsa.PublicKey) ([]byte, error) {
	if pk == nil || pk.Curve != elliptic.P256() {
		return nil, fmt.Errorf("unsupported public key (expect P-256)")
	}
	xy := make([]byte, 64)
	if !put32(xy[:32], pk.X) || !put32(xy[32:], pk.Y) {
		return nil, fmt.Errorf("x509: invalid elliptic curve public key")
	}
	return xy, nil
}

func orDefault(v, d int) int {
	if v == 0 {
		return d
	}
	return v
}

func ptr(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

func u32p(v []uint32) *C.uint32_t { return (*C.uint32_t)(unsafe.Pointer(&v[0])) }

func u8p(v []byte) *C.uint8_t { return (*C.uint8_t)(unsafe.Pointer(&v[0])) }

func cBool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}
