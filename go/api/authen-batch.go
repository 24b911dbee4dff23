// Batch verification interfaces for the MinBFT core (a new file for package
// api of the reference, next to api/api.go).  Not built in this image (no Go
// toolchain); see INTEGRATION.md §3.  Go 1.11 compatible (go.mod:30).

package api

// AuthenCall is one Authenticator.VerifyMessageAuthenTag call
// (api/api.go:133-144): the arguments the validators pass, in the same
// meaning (role, signer id, the message's AuthenBytes, the tag bytes).
type AuthenCall struct {
	Role AuthenticationRole
	ID   uint32
	Msg  []byte
	Tag  []byte
}

// Message types of AuthenMessage (the messages the core's validators see,
// core/message-handling.go:409-424, plus the REPLY).
const (
	AuthenRequest       uint32 = 1
	AuthenReply         uint32 = 2
	AuthenPrepare       uint32 = 3
	AuthenCommit        uint32 = 4
	AuthenReqViewChange uint32 = 5
)

// AuthenMessage is the authenticated content of one received message as
// raw fields -- what messages.AuthenBytes (messages/authen.go:27-76) is
// built from, plus the signature and the UIs the validators check -- so
// that an authenticator can build the AuthenBytes, hash them and verify the
// tags itself, in bulk.  No field is hashed by the caller.
//
//	REQUEST          ClientID, Seq, Op (the operation), Sig
//	REPLY            ReplicaID, ClientID, Seq, Op (the result), Sig
//	PREPARE          ReplicaID, View, and the embedded REQUEST's ClientID,
//	                 Seq, Op, Sig; UICounter / UICert (its UI)
//	COMMIT           ReplicaID, PrepReplicaID, View, the REQUEST's fields,
//	                 PrepUICounter / PrepUICert (the embedded PREPARE's UI),
//	                 UICounter / UICert (the COMMIT's own UI)
//	REQ-VIEW-CHANGE  ReplicaID, View (= the new view)
//
// The slices are borrowed for the call only.
type AuthenMessage struct {
	Type          uint32
	ReplicaID     uint32
	PrepReplicaID uint32
	ClientID      uint32
	View          uint64
	Seq           uint64
	Op            []byte
	Sig           []byte
	UICounter     uint64
	UICert        []byte
	PrepUICounter uint64
	PrepUICert    []byte
}

// MessageBatchChecker is implemented by authenticators that can run every
// signature check of a batch of messages at once (the core's validators:
// core/request.go:146-150, prepare.go:46-65, commit.go:74-92; n is the
// number of replicas, for isPrimary).  CheckMessages touches no state; each
// message is then validated by CheckedMessages.Resolve, which returns
// exactly what the core's messageValidator would return for it at that
// moment (nil, its error, or the panic it would raise) and applies the
// authenticator's state change (the USIG epoch capture, sample/
// authentication/crypto.go:219-236) only then.  The core installs its
// batched stream loop when its Stack implements this interface
// (core/message-handling-batch.go).  CheckMessages may be called
// concurrently; each CheckedMessages is used by one goroutine.
type MessageBatchChecker interface {
	CheckMessages(msgs []AuthenMessage, n uint32) (CheckedMessages, error)
}

// CheckedMessages is a batch checked by MessageBatchChecker.
type CheckedMessages interface {
	// Resolve validates message i of the batch now (see above).
	Resolve(i int) error
	// Close releases the batch; messages not resolved were never validated.
	Close()
}

// ReplyBatchVerifier is implemented by authenticators that can check a
// batch of REPLY messages a client has received at once (the client's
// replyAuthenticator, client/message-handling.go:159-170: ClientID first,
// then VerifyMessageAuthenTag(ReplicaAuthen, ...)).  The replies are
// AuthenMessages of Type AuthenReply (ReplicaID, ClientID, Seq, Op = the
// result, Sig).  CheckReplies touches no state (ReplicaAuthen has none);
// the client's reply loop (client/message-handling-batch.go) then takes
// each REPLY's verdict in order.  CheckReplies may be called concurrently.
type ReplyBatchVerifier interface {
	CheckReplies(replies []AuthenMessage, clientID uint32) (CheckedReplies, error)
}

// CheckedReplies is a batch checked by ReplyBatchVerifier.
type CheckedReplies interface {
	// Result returns exactly what the client's replyAuthenticator returns for
	// REPLY i -- nil, "Client ID mismatch" or the authenticator's error --
	// or raises the panic it would raise (a malformed DER signature,
	// sample/authentication/crypto.go:82-84).
	Result(i int) error
}
