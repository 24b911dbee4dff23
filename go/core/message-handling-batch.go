// Batched stream loop for the MinBFT core (a new file for package minbft of
// the reference, next to core/message-handling.go).  Not built in this image
// (no Go toolchain); see INTEGRATION.md §3.  Go 1.11 compatible (go.mod:30).
//
// The reference loop (core/message-handling.go:204-246) takes one message
// off the stream, unmarshals it, validates it (1 to 3 authenticator calls,
// core/request.go:146-150, prepare.go:46-65, commit.go:74-92) and processes
// it, and ends the stream at the first error.  This form takes every
// message already received (up to maxBatch), hands their raw authenticated
// fields to the authenticator's CheckMessages -- AuthenBytes, SHA-256,
// DER / UI decode and every signature of the batch on the GPU in one round
// trip; nothing is hashed here -- and then runs the UNCHANGED per-message
// path (handleMessage) in order.  The message validator (wrapped by
// withBatchVerdict) finds the message's checked verdict and resolves it at
// that moment: the USIG epoch step happens in exactly the reference's
// sequence, a reject still ends the stream at that message, a panic still
// panics there, and a message after one that failed (in validation or in
// processing) is never validated.
//
// Wiring (INTEGRATION.md §3): core/replica.go:84-85 and
// core/message-handling.go:258 call makeStreamHandler instead of
// makeMessageStreamHandler, and defaultMessageHandlers wraps its message
// and request validators with withBatchVerdict / withBatchRequestVerdict.
// makeStreamHandler picks this loop when the Stack implements
// api.MessageBatchChecker (api/authen-batch.go) and the reference loop
// otherwise.  The core imports nothing from sample/.
package minbft

import (
	"fmt"
	"sync"

	logging "github.com/op/go-logging"

	"github.com/hyperledger-labs/minbft/api"
	"github.com/hyperledger-labs/minbft/messages"
)

// maxBatch bounds the messages one CheckMessages covers.
const maxBatch = 4096

// makeStreamHandler returns the batched stream loop when stack can check
// message batches, else the reference loop.  stack is the Stack the replica
// was built with (for startPeerConnections, the same value seen as its
// api.ReplicaConnector); n is the number of replicas.
func makeStreamHandler(stack interface{}, n uint32, handleMessage messageHandler, remote string,
	logger *logging.Logger) messageStreamHandler {
	if c, ok := stack.(api.MessageBatchChecker); ok {
		return makeBatchedMessageStreamHandler(handleMessage, c, n, remote, logger)
	}
	return makeMessageStreamHandler(handleMessage, remote, logger)
}

// authenMessage extracts the raw authenticated fields of msg (the inputs of
// messages.AuthenBytes, messages/authen.go:52-76, and the tags the
// validators check); false for a message the validators do not see (Hello)
// or cannot take as is.
func authenMessage(msg messages.Message) (api.AuthenMessage, bool) {
	switch m := msg.(type) {
	case messages.Request:
		return api.AuthenMessage{Type: api.AuthenRequest, ClientID: m.ClientID(), Seq: m.Sequence(),
			Op: m.Operation(), Sig: m.Signature()}, true
	case messages.Reply:
		return api.AuthenMessage{Type: api.AuthenReply, ReplicaID: m.ReplicaID(), ClientID: m.ClientID(),
			Seq: m.Sequence(), Op: m.Result(), Sig: m.Signature()}, true
	case messages.Prepare:
		req, ui := m.Request(), m.UI()
		if req == nil || ui == nil {
			return api.AuthenMessage{}, false
		}
		return api.AuthenMessage{Type: api.AuthenPrepare, ReplicaID: m.ReplicaID(), View: m.View(),
			ClientID: req.ClientID(), Seq: req.Sequence(), Op: req.Operation(), Sig: req.Signature(),
			UICounter: ui.Counter, UICert: ui.Cert}, true
	case messages.Commit:
		prep, ui := m.Prepare(), m.UI()
		if prep == nil || ui == nil || prep.Request() == nil || prep.UI() == nil {
			return api.AuthenMessage{}, false
		}
		req, pui := prep.Request(), prep.UI()
		return api.AuthenMessage{Type: api.AuthenCommit, ReplicaID: m.ReplicaID(),
			PrepReplicaID: prep.ReplicaID(), View: prep.View(), ClientID: req.ClientID(),
			Seq: req.Sequence(), Op: req.Operation(), Sig: req.Signature(), UICounter: ui.Counter,
			UICert: ui.Cert, PrepUICounter: pui.Counter, PrepUICert: pui.Cert}, true
	case messages.ReqViewChange:
		return api.AuthenMessage{Type: api.AuthenReqViewChange, ReplicaID: m.ReplicaID(),
			View: m.NewView()}, true
	}
	return api.AuthenMessage{}, false
}

// batchVerdicts: the checked batch and index of each message the batched
// loop is handing to its handler.  Keyed by the message value the loop
// unmarshalled (a pointer: one entry per received message, never an
// embedded one), so the validator the handler calls finds exactly it.
var batchVerdicts = struct {
	sync.Mutex
	m map[messages.Message]verdictRef
}{m: make(map[messages.Message]verdictRef)}

type verdictRef struct {
	batch api.CheckedMessages
	i     int
}

func putVerdict(msg messages.Message, b api.CheckedMessages, i int) {
	batchVerdicts.Lock()
	batchVerdicts.m[msg] = verdictRef{b, i}
	batchVerdicts.Unlock()
}

func takeVerdict(msg messages.Message) (verdictRef, bool) {
	batchVerdicts.Lock()
	defer batchVerdicts.Unlock()
	v, ok := batchVerdicts.m[msg]
	if ok {
		delete(batchVerdicts.m, msg)
	}
	return v, ok
}

// withBatchVerdict wraps the replica's message validator
// (core/message-handling.go:409-424): a message the batched loop checked is
// resolved from its batch (the same nil / error / panic as validate), any
// other message is validated by validate itself.
func withBatchVerdict(validate messageValidator) messageValidator {
	return func(msg messages.Message) error {
		if v, ok := takeVerdict(msg); ok {
			return v.batch.Resolve(v.i)
		}
		return validate(msg)
	}
}

// withBatchRequestVerdict is withBatchVerdict for the client stream's
// request validator (core/message-handling.go:379-405, request.go:146-150).
func withBatchRequestVerdict(validate requestValidator) requestValidator {
	return func(req messages.Request) error {
		if v, ok := takeVerdict(req); ok {
			return v.batch.Resolve(v.i)
		}
		return validate(req)
	}
}

// readAhead moves the stream's messages, as they arrive, from the
// transport's channel (unbuffered: sample/conn/grpc/server/server.go:89,97,
// core/message-handling.go:270) into a buffered one, so that a batch sees
// every message already received.  Same messages, same order; it stops when
// `in` closes or the loop has ended (done).  Once done is closed it reads
// nothing more from `in` (as the reference loop, which simply returns), except
// at most the one message a receive racing with the close may take, which is
// dropped.
func readAhead(in <-chan []byte, done <-chan struct{}) <-chan []byte {
	q := make(chan []byte, maxBatch)
	go func() {
		defer close(q)
		for {
			select { // done first: a closed done wins over a waiting message
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

// makeBatchedMessageStreamHandler is makeMessageStreamHandler with every
// message already received checked as one GPU batch.
func makeBatchedMessageStreamHandler(handleMessage messageHandler, checker api.MessageBatchChecker,
	n uint32, remote string, logger *logging.Logger) messageStreamHandler {
	return func(in <-chan []byte, out chan<- []byte) {
		done := make(chan struct{})
		defer close(done)
		q := readAhead(in, done)
		for first := range q {
			raw := [][]byte{first}
		drain:
			for len(raw) < maxBatch {
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
			// unmarshal in order; a failure ends the stream at that message
			// (message-handling.go:207-211), after the ones before it
			msgs := make([]messages.Message, 0, len(raw))
			var parseErr error
			for _, b := range raw {
				m, err := messageImpl.NewFromBinary(b)
				if err != nil {
					parseErr = err
					break
				}
				msgs = append(msgs, m)
			}
			if !handleBatch(handleMessage, checker, n, msgs, remote, logger, out) {
				return
			}
			if parseErr != nil {
				logger.Warningf("Error unmarshaling message from %s: %s", remote, parseErr)
				return
			}
		}
	}
}

// handleBatch checks msgs as one batch, then handles them one by one in
// order, each validated (resolved) by the handler's validator; false ends
// the stream.  If the batch check itself fails (a GPU failure), every
// message takes the reference path (its validator calls the
// authenticator one call at a time).
func handleBatch(handleMessage messageHandler, checker api.MessageBatchChecker, n uint32,
	msgs []messages.Message, remote string, logger *logging.Logger, out chan<- []byte) bool {
	fields := make([]api.AuthenMessage, 0, len(msgs))
	rec := make([]int, len(msgs))
	for i, m := range msgs {
		rec[i] = -1
		if f, ok := authenMessage(m); ok {
			rec[i] = len(fields)
			fields = append(fields, f)
		}
	}
	var checked api.CheckedMessages
	if len(fields) > 0 {
		c, err := checker.CheckMessages(fields, n)
		if err != nil {
			logger.Warningf("Batch check of %d messages from %s failed, validating one by one: %s",
				len(fields), remote, err)
		} else {
			checked = c
			defer c.Close()
		}
	}
	for i, msg := range msgs {
		if checked != nil && rec[i] >= 0 {
			putVerdict(msg, checked, rec[i])
		}
		ok := handleOne(handleMessage, msg, remote, logger, out)
		takeVerdict(msg) // not consumed if the handler did not validate it
		if !ok {
			return false
		}
	}
	return true
}

// handleOne is the body of the reference loop for one message
// (message-handling.go:213-244); false ends the stream.
func handleOne(handleMessage messageHandler, msg messages.Message, remote string,
	logger *logging.Logger, out chan<- []byte) bool {
	msgStr := messages.Stringify(msg)
	logger.Debugf("Received %s from %s", msgStr, remote)
	replyChan, new, err := handleMessage(msg)
	if err != nil {
		logger.Warningf("Error handling %s from %s: %s", msgStr, remote, err)
		return false
	} else if !new {
		logger.Debugf("Dropped %s from %s", msgStr, remote)
	} else {
		logger.Debugf("Handled %s from %s", msgStr, remote)
	}
	if replyChan != nil {
		remote := remote // avoid data race with logger
		switch m := msg.(type) {
		case messages.Hello:
			remote = fmt.Sprintf("replica %d", m.ReplicaID())
		case messages.ClientMessage:
			remote = fmt.Sprintf("client %d", m.ClientID())
		}
		for m := range replyChan {
			logger.Debugf("Sending %s to %s", messages.Stringify(m), remote)
			replyBytes, err := m.MarshalBinary()
			if err != nil {
				panic(err)
			}
			out <- replyBytes
		}
	}
	return true
}
