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
//   - Prefetch: the pure part of n calls (all signatures) on the GPU now, no
//     state touched; later VerifyMessageAuthenTag calls on the same bytes
//     resolve on the host in their own order (mbft_resolve_checked).  This is
//     what the batched core stream loop (../core/message-handling-batch.go)
//     uses: the core keeps its per-message, per-stream order and its code.
//
// Swap point: sample/peer/cmd/run.go:104 (authen.NewWithSGXUSIG ->
// gpuauth.New), core/integration_test.go:154 for the in-process test.
//
// cgo pointer rules: batches are marshalled into library-owned page-locked
// C memory (mbft_host_alloc; the GPU then decodes them); single calls pass
// Go memory only as direct arguments (mbft_verify_message_authen_tag,
// mbft_resolve_checked), never stored in C memory, so the package is clean
// under GODEBUG=cgocheck=2.
//
// This package is written against the C-ABI and is not built in this
// repository's image (no Go toolchain); see INTEGRATION.md.
package gpuauth

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../minbft_amd -lminbft_amd -Wl,-rpath,${SRCDIR}/../../minbft_amd
#include <stdlib.h>
#include "minbft_gpu.h"
*/
import "C"

import (
	"crypto/ecdsa"
	"crypto/elliptic"
	"crypto/sha256"
	"encoding/binary"
	"fmt"
	"sync"
	"unsafe"

	"github.com/hyperledger-labs/minbft/api"
)

// Config selects the devices and the comb-table windows (include/minbft_gpu.h:
// HBM cost per window).  Zero values take the defaults below.
type Config struct {
	// Devices: the first builds the context, every other one gets an engine
	// with replicas of all tables; host batches are sharded across them
	// (no collective).  Default {0}.
	Devices []int
	// Windows in bits (4..29).  Defaults: generator 26, replicas and USIG
	// keys 22 (a static replica set), clients 16 (many keys).
	GeneratorWindow, ReplicaWindow, USIGWindow, ClientWindow int
	// Private keys of the ECDSA roles this node signs as
	// (GenerateMessageAuthenTag, crypto.go:63-76).
	PrivateKeys map[api.AuthenticationRole]*ecdsa.PrivateKey
	// USIGGenerator generates USIG UIs: the reference authenticator built
	// by authen.NewWithSGXUSIG (generation stays in the SGX enclave).
	USIGGenerator api.Authenticator
	// PrefetchCacheMax bounds the prefetched-verdict cache (default 1<<20).
	PrefetchCacheMax int
	// Coalesce verifies concurrent VerifyMessageAuthenTag calls (goroutines)
	// together: calls arriving while a batch is on the GPU share the next
	// one (mbft_set_coalescing).  CoalesceWaitMicros > 0 also lets a lone
	// call wait that long for company; CoalesceMaxBatch caps a batch.
	Coalesce           bool
	CoalesceWaitMicros uint32
	CoalesceMaxBatch   uint32
}

// Authenticator implements api.Authenticator on the GPU.
type Authenticator struct {
	ctx     *C.mbft_ctx
	usigGen api.Authenticator

	mu       sync.Mutex
	cache    map[[32]byte]prefetched
	cacheMax int

	ar arena // batches are marshalled here (library page-locked memory)
}

type prefetched struct {
	pure uint8 // the call's status if its USIG epoch check passes
	uses int   // prefetched occurrences not yet consumed
}

var _ api.Authenticator = (*Authenticator)(nil)

// Call is one VerifyMessageAuthenTag call.
type Call struct {
	Role api.AuthenticationRole
	ID   uint32
	Msg  []byte
	Tag  []byte
}

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
	a := &Authenticator{ctx: ctx, usigGen: cfg.USIGGenerator,
		cache: make(map[[32]byte]prefetched), cacheMax: cfg.PrefetchCacheMax}
	if a.cacheMax == 0 {
		a.cacheMax = 1 << 20
	}
	fail := func(what string, rc C.int) (*Authenticator, error) {
		err := fmt.Errorf("%s: %d (%s)", what, int(rc), C.GoString(C.mbft_last_error(ctx)))
		a.Close()
		return nil, err
	}
	if rc := C.mbft_set_generator_window(ctx, C.int(orDefault(cfg.GeneratorWindow, 26))); rc != C.MBFT_OK {
		return fail("mbft_set_generator_window", rc)
	}
	for _, d := range devices[1:] {
		if rc := C.mbft_ctx_add_device(ctx, C.int(d)); rc != C.MBFT_OK {
			return fail(fmt.Sprintf("mbft_ctx_add_device(%d)", d), rc)
		}
	}
	for role, m := range keys {
		w := orDefault(cfg.ReplicaWindow, 22)
		switch role {
		case api.ClientAuthen:
			w = orDefault(cfg.ClientWindow, 16)
		case api.USIGAuthen:
			w = orDefault(cfg.USIGWindow, 22)
		}
		if rc := C.mbft_set_key_window(ctx, C.int(w)); rc != C.MBFT_OK {
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
		}
	}
	for role, sk := range cfg.PrivateKeys {
		d := make([]byte, 32)
		sk.D.FillBytes(d)
		if rc := C.mbft_set_private_key(ctx, C.uint32_t(role),
			(*C.uint8_t)(unsafe.Pointer(&d[0]))); rc != C.MBFT_OK {
			return fail("mbft_set_private_key", rc)
		}
	}
	C.mbft_enable_usig(ctx, cBool(usigEnabled))
	if cfg.Coalesce {
		if rc := C.mbft_set_coalescing(ctx, 1, C.uint32_t(cfg.CoalesceWaitMicros),
			C.uint32_t(cfg.CoalesceMaxBatch)); rc != C.MBFT_OK {
			return fail("mbft_set_coalescing", rc)
		}
	}
	return a, nil
}

// Close releases the GPU context and its tables.
func (a *Authenticator) Close() {
	a.ar.release()
	if a.ctx != nil {
		C.mbft_ctx_destroy(a.ctx)
		a.ctx = nil
	}
}

// VerifyMessageAuthenTag implements api.Authenticator.  A call prefetched
// with the same bytes resolves on the host (no GPU round trip); any other
// is verified as a batch of one.
func (a *Authenticator) VerifyMessageAuthenTag(role api.AuthenticationRole, id uint32,
	msg []byte, tag []byte) error {
	if pure, ok := a.takePrefetched(role, id, msg, tag); ok {
		st := C.mbft_resolve_checked(a.ctx, C.uint32_t(role), C.uint32_t(id), ptr(msg),
			C.size_t(len(msg)), ptr(tag), C.size_t(len(tag)), C.uint8_t(pure))
		return statusToErr(role, int(st))
	}
	st := C.mbft_verify_message_authen_tag(a.ctx, C.uint32_t(role), C.uint32_t(id), ptr(msg),
		C.size_t(len(msg)), ptr(tag), C.size_t(len(tag)))
	return statusToErr(role, int(st))
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
	a.ar.mu.Lock()
	defer a.ar.mu.Unlock()
	f := a.ar.flatten(calls)
	rc := C.mbft_verify_batch_flat(a.ctx, u32p(f.roles), u32p(f.ids), ptr(f.msgs), u64p(f.msgOff),
		ptr(f.tags), u64p(f.tagOff), C.size_t(n), ptr(f.status))
	if rc != C.MBFT_OK {
		panic(fmt.Sprintf("mbft_verify_batch_flat: %d (%s)", int(rc), C.GoString(C.mbft_last_error(a.ctx))))
	}
	for i := range calls {
		out[i] = statusToErr(calls[i].Role, int(f.status[i]))
	}
	return out
}

// Prefetch checks the pure part of calls on the GPU (every signature, no
// USIG epoch state) and keeps the verdicts for the VerifyMessageAuthenTag
// calls that will repeat them, in whatever order the caller makes them.
func (a *Authenticator) Prefetch(calls []Call) {
	n := len(calls)
	if n == 0 {
		return
	}
	a.ar.mu.Lock()
	f := a.ar.flatten(calls)
	rc := C.mbft_check_batch_flat(a.ctx, u32p(f.roles), u32p(f.ids), ptr(f.msgs), u64p(f.msgOff),
		ptr(f.tags), u64p(f.tagOff), C.size_t(n), ptr(f.status))
	pure := append([]byte(nil), f.status...)
	a.ar.mu.Unlock()
	if rc != C.MBFT_OK {
		return // the calls simply go to the GPU one by one later
	}
	a.mu.Lock()
	defer a.mu.Unlock()
	if len(a.cache)+n > a.cacheMax {
		a.cache = make(map[[32]byte]prefetched) // stale predictions: drop them
	}
	for i, c := range calls {
		k := callKey(c.Role, c.ID, c.Msg, c.Tag)
		e := a.cache[k]
		e.pure = pure[i]
		e.uses++
		a.cache[k] = e
	}
}

func (a *Authenticator) takePrefetched(role api.AuthenticationRole, id uint32, msg, tag []byte) (uint8, bool) {
	k := callKey(role, id, msg, tag)
	a.mu.Lock()
	defer a.mu.Unlock()
	e, ok := a.cache[k]
	if !ok {
		return 0, false
	}
	if e.uses--; e.uses <= 0 {
		delete(a.cache, k)
	} else {
		a.cache[k] = e
	}
	return e.pure, true
}

// GenerateMessageAuthenTag implements api.Authenticator: the ECDSA roles
// sign on the GPU (Sum(m) digest, DER, crypto.go:63-76,113-116); the USIG
// role goes to the SGX-backed reference authenticator.
func (a *Authenticator) GenerateMessageAuthenTag(role api.AuthenticationRole,
	msg []byte) ([]byte, error) {
	if role == api.USIGAuthen {
		if a.usigGen == nil {
			return nil, fmt.Errorf("no USIG to generate UIs")
		}
		return a.usigGen.GenerateMessageAuthenTag(role, msg)
	}
	buf := make([]byte, 80)
	var n C.size_t
	rc := C.mbft_generate_message_authen_tag(a.ctx, C.uint32_t(role), ptr(msg), C.size_t(len(msg)),
		(*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(len(buf)), &n)
	if rc != C.MBFT_OK {
		return nil, fmt.Errorf("failed to generate authentication tag: %d", int(rc))
	}
	return buf[:n], nil
}

// ---------------------------------------------------------------- helpers

type flat struct {
	roles, ids         []uint32
	msgs, tags, status []byte
	msgOff, tagOff     []uint64
}

// arena: library-owned page-locked host memory (mbft_host_alloc) the batches
// are marshalled into.  It is C memory, so passing it is clean under the cgo
// pointer rules, and a batch whose buffers all lie in it travels to the GPU
// raw and is decoded there (DER, digest, key; include/minbft_gpu.h): the
// library's host threads read none of its bytes.  Grown on demand, reused
// across batches, guarded by mu for the length of a call.
type arena struct {
	mu   sync.Mutex
	base unsafe.Pointer
	size int
}

func (ar *arena) release() {
	ar.mu.Lock()
	defer ar.mu.Unlock()
	if ar.base != nil {
		C.mbft_host_free(ar.base)
		ar.base, ar.size = nil, 0
	}
}

func (ar *arena) ensure(bytes int) bool {
	if bytes <= ar.size {
		return true
	}
	if ar.base != nil {
		C.mbft_host_free(ar.base)
		ar.base, ar.size = nil, 0
	}
	want := bytes + bytes/4
	var p unsafe.Pointer
	if C.mbft_host_alloc(C.size_t(want), &p) != C.MBFT_OK {
		return false
	}
	ar.base, ar.size = p, want
	return true
}

// flatten packs calls into the arena (8-byte aligned regions: offsets,
// roles, ids, message bytes, tag bytes, statuses); with no arena memory it
// falls back to pointer-free Go slices (passed as arguments, never retained
// by the library; decoded on the host).
func (ar *arena) flatten(calls []Call) flat {
	n := len(calls)
	var ml, tl int
	for _, c := range calls {
		ml += len(c.Msg)
		tl += len(c.Tag)
	}
	al := func(x int) int { return (x + 7) &^ 7 }
	var f flat
	if ar.ensure(2*al(8*(n+1)) + 2*al(4*n) + al(ml+1) + al(tl+1) + al(n)) {
		b := unsafe.Slice((*byte)(ar.base), ar.size)
		o := 0
		take := func(sz int) unsafe.Pointer {
			p := unsafe.Pointer(&b[o])
			o += al(sz)
			return p
		}
		f.msgOff = unsafe.Slice((*uint64)(take(8*(n+1))), n+1)
		f.tagOff = unsafe.Slice((*uint64)(take(8*(n+1))), n+1)
		f.roles = unsafe.Slice((*uint32)(take(4*n)), n)
		f.ids = unsafe.Slice((*uint32)(take(4*n)), n)
		f.msgs = unsafe.Slice((*byte)(take(ml+1)), ml+1)
		f.tags = unsafe.Slice((*byte)(take(tl+1)), tl+1)
		f.status = unsafe.Slice((*byte)(take(n)), n)
	} else {
		f = flat{roles: make([]uint32, n), ids: make([]uint32, n), msgs: make([]byte, ml+1),
			tags: make([]byte, tl+1), status: make([]byte, n),
			msgOff: make([]uint64, n+1), tagOff: make([]uint64, n+1)}
	}
	var mo, to int
	f.msgOff[0], f.tagOff[0] = 0, 0
	for i, c := range calls {
		f.roles[i] = uint32(c.Role)
		f.ids[i] = c.ID
		mo += copy(f.msgs[mo:], c.Msg)
		to += copy(f.tags[to:], c.Tag)
		f.msgOff[i+1] = uint64(mo)
		f.tagOff[i+1] = uint64(to)
	}
	return f
}

func callKey(role api.AuthenticationRole, id uint32, msg, tag []byte) [32]byte {
	h := sha256.New()
	var hdr [16]byte
	binary.BigEndian.PutUint32(hdr[0:], uint32(role))
	binary.BigEndian.PutUint32(hdr[4:], id)
	binary.BigEndian.PutUint64(hdr[8:], uint64(len(msg)))
	h.Write(hdr[:])
	h.Write(msg)
	h.Write(tag)
	var k [32]byte
	copy(k[:], h.Sum(nil))
	return k
}

func rawXY(pk *ecdsa.PublicKey) ([]byte, error) {
	if pk == nil || pk.Curve != elliptic.P256() {
		return nil, fmt.Errorf("unsupported public key (expect P-256)")
	}
	xy := make([]byte, 64)
	pk.X.FillBytes(xy[:32])
	pk.Y.FillBytes(xy[32:])
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

func u64p(v []uint64) *C.uint64_t { return (*C.uint64_t)(unsafe.Pointer(&v[0])) }

func cBool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}
