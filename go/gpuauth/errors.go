package gpuauth

/*
#include "minbft_gpu.h"
*/
import "C"

import (
	"fmt"

	"github.com/hyperledger-labs/minbft/api"
)

// statusToErr maps an mbft_status to the reference's outcome: nil, an error
// with the reference's text where one status has one text, or the panic of
// EcdsaSigCipher.Verify on malformed DER in an ECDSA role (crypto.go:82-84).
// The texts are log-only in the core (core/message-handling.go:217-218);
// the nil / error / panic outcome is what the tests pin.
//
//   - ECDSA roles: the scheme's only error is "invalid signature"
//     (crypto.go:120-126), wrapped by authenticator.go:130-132 -- also for an
//     unknown id, whose nil key makes EcdsaSigCipher.Verify return false
//     (crypto.go:85-88).
//   - USIG role: the texts of crypto.go:186-239, usig/sgx/sgx-usig.go:81-97
//     and usig/sgx/usig-enclave.go:198-229, wrapped the same way.
//   - MBFT_UNKNOWN_ROLE covers two reference errors that are not wrapped:
//     no key set for the role (keymanager.go:96-101) and a key set without
//     a scheme (authenticator.go:126-129); the first is the one a replica
//     meets (a role missing from keys.yaml).
//
// Negative values are C-ABI failures (HIP error, out of memory): the
// reference cannot fail that way.  Policy (INTEGRATION.md §2): the binding
// retries the C call once; if it fails again the call is REJECTED with an
// error naming the failure (Authenticator.failure).  Never accepted: a GPU
// failure cannot make a forged message pass, and the replica keeps running
// (the core ends that one stream, as for any reject,
// core/message-handling.go:217-220) instead of crashing as a panic would.
// The library leaves no partial state behind a failed call (its streams are
// drained, the USIG epoch state is only written after every signature of a
// batch is checked; tests/test_gpu_failures.py).
func (a *Authenticator) statusToErr(role api.AuthenticationRole, id uint32, st int) error {
	if st < 0 {
		return a.failure("mbft_verify_message_authen_tag", st)
	}
	return statusToErr(role, id, st)
}

// failure is the error of a call whose C-ABI call failed twice.
func (a *Authenticator) failure(what string, rc int) error {
	return fmt.Errorf("GPU authenticator failure: %s: %d (%s)", what, rc,
		C.GoString(C.mbft_last_error(a.ctx)))
}

func statusToErr(role api.AuthenticationRole, id uint32, st int) error {
	if st < 0 {
		return fmt.Errorf("GPU authenticator failure: %d", st)
	}
	usig := role == api.USIGAuthen
	switch st {
	case C.MBFT_ACCEPT:
		return nil
	case C.MBFT_MALFORMED_DER:
		if !usig {
			panic("ECDSA signature is not ASN.1-DER encoded: asn1: structure error") // crypto.go:82-84
		}
		return tagError("failed to unmarshal USIG signature: asn1: structure error") // usig-enclave.go:217-219
	case C.MBFT_REJECT_SIG:
		if usig {
			return tagError("signature not valid") // usig-enclave.go:224-226
		}
		return tagError("invalid signature") // crypto.go:122-124
	case C.MBFT_UNKNOWN_KEY:
		if usig {
			return tagError("Failed to calculate USIG key fingerprint: x509: unsupported public key type: <nil>") // crypto.go:192-195
		}
		return tagError("invalid signature") // nil key: Verify returns false (crypto.go:85-88)
	case C.MBFT_DER_TRAILING:
		return tagError("extra bytes in USIG signature") // usig-enclave.go:220-221
	case C.MBFT_BAD_KEY:
		return tagError("invalid public key")
	case C.MBFT_BAD_UI:
		return tagError("failed to unmarshal UI: unexpected EOF") // crypto.go:189-191, usig/usig.go:72-78
	case C.MBFT_BAD_CERT:
		return tagError("failed to parse UI cert: failed to extract epoch from USIG cert: unexpected EOF") // sgx-usig.go:86-90,162-165
	case C.MBFT_EPOCH_MISMATCH:
		return tagError("epoch value mismatch") // sgx-usig.go:92-94
	case C.MBFT_UNKNOWN_ROLE:
		return fmt.Errorf("key set not found for role=%v, id=%d", role, id) // keymanager.go:96-101
	}
	return tagError(fmt.Sprintf("status %d", st))
}

func tagError(why string) error {
	return fmt.Errorf("Invalid authentication tag: %s", why) // authenticator.go:130-132
}
