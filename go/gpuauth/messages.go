package gpuauth

// api.MessageBatchChecker on the GPU: a batch of received messages goes to
// the library as records + one byte arena in page-locked C memory
// (mbft_msg_rec, include/minbft_gpu.h) -- raw fields only, nothing hashed in
// Go -- and mbft_check_messages_flat runs the validators' pure part there:
// AuthenBytes (messages/authen.go:27-76), SHA-256, the Sum(m) quirk and the
// USIG digest chain, DER and UI decode, key lookups and every signature.
// MessageBatch.Resolve then validates one message in the core's order
// (mbft_resolve_message: the USIG epoch step, crypto.go:219-236, applied at
// that moment) and maps its result to what the core's messageValidator
// returns: nil, the validator's error, or its panic.

/*
#include "minbft_gpu.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	"github.com/hyperledger-labs/minbft/api"
)

// msgInfo keeps what a result's error text needs of each message.
type msgInfo struct {
	typ, replica, primary, client uint32
	view                          uint64
}

// MessageBatch is a batch checked by CheckMessages (api.CheckedMessages).
type MessageBatch struct {
	a    *Authenticator
	b    *C.mbft_msg_batch
	info []msgInfo
}

var _ api.CheckedMessages = (*MessageBatch)(nil)

// maxRecs: the largest record array the pre-Go-1.17 slice idiom addresses.
const maxRecs = 1 << 26

// CheckMessages implements api.MessageBatchChecker (n: the number of
// replicas, for isPrimary).  The signers' keys are made present first
// (keys.go), so every status is the one the reference gives.
func (a *Authenticator) CheckMessages(msgs []api.AuthenMessage, n uint32) (api.CheckedMessages, error) {
	if len(msgs) > maxRecs {
		return nil, fmt.Errorf("batch of %d messages: more than %d", len(msgs), maxRecs)
	}
	a.ensureMessageKeys(msgs)
	ar := a.arenas.get()
	defer a.arenas.put(ar)
	recs, bytes, nbytes := ar.packMessages(msgs)
	var b *C.mbft_msg_batch
	rc := C.mbft_check_messages_flat(a.ctx, recs, C.size_t(len(msgs)), bytes, C.size_t(nbytes),
		C.uint32_t(n), &b)
	if rc < 0 { // once more (errors.go); a failed check touched no state
		rc = C.mbft_check_messages_flat(a.ctx, recs, C.size_t(len(msgs)), bytes, C.size_t(nbytes),
			C.uint32_t(n), &b)
	}
	if rc != C.MBFT_OK {
		return nil, a.failure("mbft_check_messages_flat", int(rc))
	}
	mb := &MessageBatch{a: a, b: b, info: make([]msgInfo, len(msgs))}
	for i, m := range msgs {
		mb.info[i] = msgInfo{typ: m.Type, replica: m.ReplicaID, primary: m.PrepReplicaID,
			client: m.ClientID, view: m.View}
	}
	return mb, nil
}

// Resolve implements api.CheckedMessages: message i validated now.
func (mb *MessageBatch) Resolve(i int) error {
	r := C.mbft_resolve_message(mb.a.ctx, mb.b, C.size_t(i))
	if r < 0 {
		return mb.a.failure("mbft_resolve_message", int(r))
	}
	return messageError(mb.info[i], int(r))
}

// Close implements api.CheckedMessages.
func (mb *MessageBatch) Close() {
	if mb.b != nil {
		C.mbft_msg_batch_free(mb.b)
		mb.b = nil
	}
}

// ensureMessageKeys registers late keys (keys.go) for every signer of the
// batch: the REQUEST's client, the PREPARE's and COMMIT's USIG instances.
func (a *Authenticator) ensureMessageKeys(msgs []api.AuthenMessage) {
	if a.keys.ks == nil {
		return
	}
	var calls []Call
	for _, m := range msgs {
		switch m.Type {
		case api.AuthenRequest, api.AuthenPrepare, api.AuthenCommit:
			calls = append(calls, Call{Role: api.ClientAuthen, ID: m.ClientID})
		}
		switch m.Type {
		case api.AuthenPrepare:
			calls = append(calls, Call{Role: api.USIGAuthen, ID: m.ReplicaID})
		case api.AuthenCommit:
			calls = append(calls, Call{Role: api.USIGAuthen, ID: m.PrepReplicaID},
				Call{Role: api.USIGAuthen, ID: m.ReplicaID})
		case api.AuthenReply:
			calls = append(calls, Call{Role: api.ReplicaAuthen, ID: m.ReplicaID})
		}
	}
	a.ensureKeys(calls)
}

// packMessages marshals msgs into the arena: the records (mbft_msg_rec, 104
// bytes each), then every variable field back to back, addressed by offsets
// into that byte region.  Without arena memory it uses Go slices (legal cgo
// arguments: the records hold no pointers; the library stages them into
// its own page-locked memory).
func (ar *arena) packMessages(msgs []api.AuthenMessage) (*C.mbft_msg_rec, *C.uint8_t, int) {
	n := len(msgs)
	nb := 0
	for i := range msgs {
		m := &msgs[i]
		nb += len(m.Op) + len(m.Sig) + len(m.UICert) + len(m.PrepUICert)
	}
	recBytes := (n*int(unsafe.Sizeof(C.mbft_msg_rec{})) + 7) &^ 7
	if !ar.ensure(recBytes + nb + 8) {
		// no page-locked memory: Go memory (the library stages it)
		recs := make([]C.mbft_msg_rec, n+1)
		bytes := make([]byte, nb+1)
		fillMessages(msgs, recs[:n], bytes)
		return &recs[0], (*C.uint8_t)(unsafe.Pointer(&bytes[0])), nb
	}
	recs := (*[maxRecs]C.mbft_msg_rec)(ar.base)[:n:n]
	bytes := bytesAt(arenaAt(ar.base, recBytes), nb+1)
	fillMessages(msgs, recs, bytes)
	return (*C.mbft_msg_rec)(ar.base), (*C.uint8_t)(arenaAt(ar.base, recBytes)), nb
}

func fillMessages(msgs []api.AuthenMessage, recs []C.mbft_msg_rec, bytes []byte) {
	pos := 0
	put := func(b []byte) (C.uint64_t, C.uint32_t) {
		off := pos
		pos += copy(bytes[pos:], b)
		return C.uint64_t(off), C.uint32_t(len(b))
	}
	for i := range msgs {
		m := &msgs[i]
		r := &recs[i]
		r._type = C.uint32_t(m.Type)
		r.stream = 0
		r.replica_id = C.uint32_t(m.ReplicaID)
		r.prep_replica_id = C.uint32_t(m.PrepReplicaID)
		r.client_id = C.uint32_t(m.ClientID)
		r.reserved = 0
		r.view = C.uint64_t(m.View)
		r.seq = C.uint64_t(m.Seq)
		r.ui_counter = C.uint64_t(m.UICounter)
		r.prep_ui_counter = C.uint64_t(m.PrepUICounter)
		r.op_off, r.op_len = put(m.Op)
		r.sig_off, r.sig_len = put(m.Sig)
		r.ui_cert_off, r.ui_cert_len = put(m.UICert)
		r.prep_ui_cert_off, r.prep_ui_cert_len = put(m.PrepUICert)
	}
}

// Stages of a message result (include/minbft_gpu.h enum mbft_stage).
const (
	stRequestSig        = 1
	stNotPrimary        = 2
	stPrepareUI         = 3
	stCommitFromPrimary = 4
	stCommitUI          = 5
	stNotImplemented    = 6
	stUnknownType       = 10
)

// messageError is what the core's messageValidator returns for a message
// with result res ((stage << 8) | status, 0 = valid): the errors of
// core/request.go:146-150, prepare.go:46-65, commit.go:74-92, usig-ui.go:
// 62-77 and message-handling.go:409-424 around the authenticator's error
// (errors.go), or their panics (crypto.go:82-84: malformed DER in the
// REQUEST's signature; message-handling.go:420-421: a message type the
// replica's validator does not know).  Texts are log-only in the core.
func messageError(m msgInfo, res int) error {
	if res == 0 {
		return nil
	}
	stage, st := res>>8, res&0xFF
	inPrepare := func(err error) error { // a COMMIT validates its PREPARE (commit.go:82-84)
		if m.typ == api.AuthenCommit {
			return fmt.Errorf("Invalid Prepare: %s", err)
		}
		return err
	}
	uiErr := func(id uint32) error { // usig-ui.go:62-77
		if st == C.MBFT_ZERO_COUNTER {
			return fmt.Errorf("Invalid (zero) counter value")
		}
		return fmt.Errorf("Failed verifying USIG certificate: %s", statusToErr(api.USIGAuthen, id, st))
	}
	switch stage {
	case stUnknownType:
		panic("Unknown message type")
	case stNotImplemented:
		return fmt.Errorf("Not implemented")
	case stRequestSig:
		err := statusToErr(api.ClientAuthen, m.client, st) // panics on malformed DER
		if m.typ == api.AuthenRequest {
			return err
		}
		return inPrepare(fmt.Errorf("Request invalid: %s", err))
	case stNotPrimary:
		replica := m.replica
		if m.typ == api.AuthenCommit {
			replica = m.primary
		}
		return inPrepare(fmt.Errorf("Prepare from backup %d for view %d", replica, m.view))
	case stPrepareUI:
		replica := m.replica
		if m.typ == api.AuthenCommit {
			replica = m.primary
		}
		return inPrepare(fmt.Errorf("UI not valid: %s", uiErr(replica)))
	case stCommitFromPrimary:
		return fmt.Errorf("Commit from primary")
	case stCommitUI:
		return fmt.Errorf("UI is not valid: %s", uiErr(m.replica))
	}
	return fmt.Errorf("validation result %#x", res)
}
