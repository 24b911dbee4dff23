// Batched stream loop for the MinBFT core (a new file for package minbft of
// the reference, next to core/message-handling.go).  Not built in this image
// (no Go toolchain); see INTEGRATION.md §3.  Go 1.11 compatible (go.mod:30).
//
// The reference loop (core/message-handling.go:204-246) takes one message
// off the stream, unmarshals it, validates it (1 to 3 authenticator calls,
// core/request.go:146-150, prepare.go:46-65, commit.go:74-92) and processes
// it, and ends the stream at the first error.  This form drains up to
// maxBatch messages that are already waiting, computes the authenticator
// calls their validators will make (same role, id, AuthenBytes and tag, in
// validator order: the REQUEST signature, the PREPARE UI, the COMMIT UI;
// zero counters are rejected before any call, usig-ui.go:65-67), hands all
// of them to the authenticator's Prefetch -- every signature checked on the
// GPU in one batch -- and then runs the UNCHANGED per-message path
// (handleMessage) in order.  Each of its VerifyMessageAuthenTag calls finds
// its prefetched verdict and resolves on the host, USIG epoch state
// included, in exactly the reference's order; a reject still ends the
// stream at that message, and messages after it are not processed.
//
// Wiring (INTEGRATION.md §3): core/replica.go:84-85 and
// core/message-handling.go:258 call makeStreamHandler instead of
// makeMessageStreamHandler; it picks this loop when the Stack implements
// api.AuthenPrefetcher (api/authen-batch.go) and the reference loop
// otherwise.  The core imports nothing from sample/.
package minbft

import (
	"fmt"

	logging "github.com/op/go-logging"

	"github.com/hyperledger-labs/minbft/api"
	"github.com/hyperledger-labs/minbft/messages"
	"github.com/hyperledger-labs/minbft/usig"
)

// maxBatch bounds the messages one Prefetch covers.
const maxBatch = 4096

// makeStreamHandler returns the batched stream loop when stack can
// prefetch authenticator verdicts, else the reference loop.  stack is the
// Stack the replica was built with (for startPeerConnections, the same
// value seen as its api.ReplicaConnector); n is the number of replicas.
func makeStreamHandler(stack interface{}, n uint32, handleMessage messageHandler, remote string,
	logger *logging.Logger) messageStreamHandler {
	if p, ok := stack.(api.AuthenPrefetcher); ok {
		return makeBatchedMessageStreamHandler(handleMessage, p, n, remote, logger)
	}
	return makeMessageStreamHandler(handleMessage, remote, logger)
}

// authenCalls lists the VerifyMessageAuthenTag calls the validators make
// for msg, in their order (n = number of replicas, for isPrimary).  Calls
// behind a check that fails without the authenticator are left out; the
// validator rejects there anyway.
func authenCalls(msg messages.Message, n uint32) []api.AuthenCall {
	var calls []api.AuthenCall
	request := func(req messages.Request) {
		calls = append(calls, api.AuthenCall{Role: api.ClientAuthen, ID: req.ClientID(),
			Msg: messages.AuthenBytes(req), Tag: req.Signature()})
	}
	ui := func(m messages.CertifiedMessage) bool {
		u := m.UI()
		if u.Counter == 0 {
			return false
		}
		calls = append(calls, api.AuthenCall{Role: api.USIGAuthen, ID: m.ReplicaID(),
			Msg: messages.AuthenBytes(m), Tag: usig.MustMarshalUI(u)})
		return true
	}
	prepare := func(prep messages.Prepare) bool {
		if !isPrimary(prep.View(), prep.ReplicaID(), n) {
			return false
		}
		request(prep.Request())
		return ui(prep)
	}
	switch m := msg.(type) {
	case messages.Request:
		request(m)
	case messages.Prepare:
		prepare(m)
	case messages.Commit:
		if m.ReplicaID() != m.Prepare().ReplicaID() && prepare(m.Prepare()) {
			ui(m)
		}
	}
	return calls
}

// makeBatchedMessageStreamHandler is makeMessageStreamHandler with the
// messages already waiting on `in` prefetched as one GPU batch.
func makeBatchedMessageStreamHandler(handleMessage messageHandler, prefetch api.AuthenPrefetcher, n uint32,
	remote string, logger *logging.Logger) messageStreamHandler {
	return func(in <-chan []byte, out chan<- []byte) {
		for first := range in {
			raw := [][]byte{first}
		drain:
			for len(raw) < maxBatch {
				select {
				case b, ok := <-in:
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
			var calls []api.AuthenCall
			for _, m := range msgs {
				calls = append(calls, authenCalls(m, n)...)
			}
			prefetch.Prefetch(calls)
			for _, msg := range msgs {
				if !handleOne(handleMessage, msg, remote, logger, out) {
					return
				}
			}
			if parseErr != nil {
				logger.Warningf("Error unmarshaling message from %s: %s", remote, parseErr)
				return
			}
		}
	}
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
