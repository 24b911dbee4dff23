package gpuauth

// api.ReplyBatchVerifier on the GPU: a client's received REPLY messages go
// to the library as records + one byte arena in page-locked C memory (the
// same marshal as messages.go: raw fields, nothing hashed in Go), and
// mbft_validate_replies_flat runs the client's replyAuthenticator on all of
// them at once (client/message-handling.go:159-170): the ClientID check,
// then ReplicaAuthen's AuthenBytes (messages/authen.go:57-60), Sum(m) digest,
// DER and signature.  A few replies take the library's small route (hashed
// on the host, one zero-copy verify launch); more, the GPU digest stage.

/*
#include "minbft_gpu.h"
*/
import "C"

import (
	"fmt"
	"unsafe"

	"github.com/hyperledger-labs/minbft/api"
)

// ReplyBatch is a batch checked by CheckReplies (api.CheckedReplies).
type ReplyBatch struct {
	res     []int32
	replica []uint32
}

var _ api.CheckedReplies = (*ReplyBatch)(nil)

// Stages of a REPLY result (include/minbft_gpu.h enum mbft_stage).
const (
	stReplySig      = 8
	stReplyClientID = 11
)

// CheckReplies implements api.ReplyBatchVerifier.  The replying replicas'
// keys are made present first (keys.go).  Every REPLY gets its own result
// (MBFT_VF_NO_PANIC_STOP): the reference panics at the first malformed
// signature when its loop reaches it, which Result(i) reproduces.
func (a *Authenticator) CheckReplies(replies []api.AuthenMessage, clientID uint32) (api.CheckedReplies, error) {
	n := len(replies)
	rb := &ReplyBatch{res: make([]int32, n), replica: make([]uint32, n)}
	if n == 0 {
		return rb, nil
	}
	if n > maxRecs {
		return nil, fmt.Errorf("batch of %d replies: more than %d", n, maxRecs)
	}
	for i := range replies {
		if replies[i].Type != api.AuthenReply {
			return nil, fmt.Errorf("CheckReplies: message %d is not a REPLY", i)
		}
		rb.replica[i] = replies[i].ReplicaID
	}
	a.ensureMessageKeys(replies)
	ar := a.arenas.get()
	defer a.arenas.put(ar)
	recs, bytes, nbytes := ar.packMessages(replies)
	out := (*C.int32_t)(unsafe.Pointer(&rb.res[0])) // (Go memory holding no pointers)
	flags := C.uint32_t(C.MBFT_VF_NO_PANIC_STOP)
	rc := C.mbft_validate_replies_flat(a.ctx, recs, C.size_t(n), bytes, C.size_t(nbytes), C.uint32_t(clientID),
		flags, out)
	if rc < 0 { // once more (errors.go); a failed check touched no state
		rc = C.mbft_validate_replies_flat(a.ctx, recs, C.size_t(n), bytes, C.size_t(nbytes),
			C.uint32_t(clientID), flags, out)
	}
	if rc != C.MBFT_OK {
		return nil, a.failure("mbft_validate_replies_flat", int(rc))
	}
	return rb, nil
}

// Result implements api.CheckedReplies.
func (rb *ReplyBatch) Result(i int) error {
	res := int(rb.res[i])
	if res == 0 {
		return nil
	}
	stage, st := res>>8, res&0xFF
	switch stage {
	case stReplyClientID:
		return fmt.Errorf("Client ID mismatch")
	case stReplySig:
		return statusToErr(api.ReplicaAuthen, rb.replica[i], st) // panics on malformed DER
	}
	return fmt.Errorf("reply result %#x", res)
}
