// Batch verification interface for the MinBFT core (a new file for package
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

// AuthenPrefetcher is implemented by authenticators that can check the
// pure part of many calls at once (every signature; no USIG epoch state is
// touched).  After Prefetch(calls), VerifyMessageAuthenTag on the same
// arguments returns exactly what it would have returned without the
// prefetch, in whatever order and from whatever goroutine it is called; a
// prefetched verdict that is never used is dropped in time.  The core
// installs its batched stream loop when its Stack implements this
// interface (core/message-handling-batch.go).  Prefetch may be called
// concurrently.  The calls' slices are borrowed for the call only.
type AuthenPrefetcher interface {
	Prefetch(calls []AuthenCall)
}
