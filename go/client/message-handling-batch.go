// The client's reply loop with batched authentication (a new file for
// package client of the reference, next to client/message-handling.go).
// Not built in this image (no Go toolchain); see INTEGRATION.md §4.  Go 1.11
// compatible (go.mod:30).

package client

import (
	"github.com/hyperledger-labs/minbft/api"
	"github.com/hyperledger-labs/minbft/messages"
)

// maxReplyBatch bounds the REPLYs authenticated in one call.
const maxReplyBatch = 1024

// makeBatchedIncomingMessageHandler is makeIncomingMessageHandler
// (client/message-handling.go:90-110) with every REPLY already received from
// the replica authenticated as one batch (api.ReplyBatchVerifier), then
// handled in arrival order exactly as makeReplyMessageHandler (:138-157)
// does: a rejected REPLY is logged and dropped, the loop goes on; a
// malformed signature panics when the loop reaches that REPLY, after every
// earlier one was handled (crypto.go:82-84).  Messages that fail to
// unmarshal or are not REPLYs are logged in place, as before.
func makeBatchedIncomingMessageHandler(replicaID, clientID uint32, verifier api.ReplyBatchVerifier,
	consumer replyConsumer) incomingMessageHandler {
	return func(in <-chan []byte) {
		done := make(chan struct{})
		defer close(done)
		q := readAheadReplies(in, done)
		for first := range q {
			raw := [][]byte{first}
		drain:
			for len(raw) < maxReplyBatch {
				select {
				case b, ok := <-q:
					if !ok {
						break drain
					}
					raw = append(raw, b)
				default:
					break drain
				}
			}
			msgs := make([]messages.Message, len(raw))
			errs := make([]error, len(raw))
			var replies []api.AuthenMessage
			at := make([]int, len(raw)) // message -> its index among the replies (-1: none)
			for i, b := range raw {
				at[i] = -1
				msgs[i], errs[i] = messageImpl.NewFromBinary(b)
				if errs[i] != nil {
					continue
				}
				if r, ok := msgs[i].(messages.Reply); ok {
					at[i] = len(replies)
					replies = append(replies, api.AuthenMessage{Type: api.AuthenReply,
						ReplicaID: r.ReplicaID(), ClientID: r.ClientID(), Seq: r.Sequence(),
						Op: r.Result(), Sig: r.Signature()})
				}
			}
			var checked api.CheckedReplies
			var cerr error
			if len(replies) > 0 {
				checked, cerr = verifier.CheckReplies(replies, clientID)
			}
			for i := range raw {
				if errs[i] != nil {
					logger.Warningf("Error unmarshaling message from replica %d: %v", replicaID, errs[i])
					continue
				}
				reply, ok := msgs[i].(messages.Reply)
				if !ok {
					logger.Warningf("Received unknown message from replica %d", replicaID)
					continue
				}
				err := cerr
				if err == nil {
					err = checked.Result(at[i]) // (the panic of crypto.go:82-84 is raised here)
				}
				handleCheckedReply(reply, err, consumer)
			}
		}
	}
}

// handleCheckedReply is makeReplyMessageHandler's body with the
// authenticator's verdict given.
func handleCheckedReply(reply messages.Reply, err error, consumer replyConsumer) {
	replicaID := reply.ReplicaID()
	if err != nil {
		logger.Warningf("Failed to authenticate Reply message from replica %d: %v", replicaID, err)
		return
	}
	logger.Debugf("Received Reply message from replica %d", replicaID)
	if ok := consumer(reply); !ok {
		logger.Infof("Dropped Reply message from replica %d", replicaID)
	}
}

// readAheadReplies moves the replica's messages, as they arrive, into a
// buffered channel so that a batch sees every message already received;
// same messages, same order; it stops when `in` closes or the loop has
// ended (done), reading nothing more from `in` after done except at most
// the one message a receive racing with the close takes.
func readAheadReplies(in <-chan []byte, done <-chan struct{}) <-chan []byte {
	q := make(chan []byte, maxReplyBatch)
	go func() {
		defer close(q)
		for {
			select {
			case <-done:
				return
			default:
			}
			select {
			case <-done:
				return
			case b, ok := <-in:
				if !ok {
					return
				}
				select {
				case q <- b:
				case <-done:
					return
				}
			}
		}
	}()
	return q
}
