package gpuauth

/*
#include "minbft_gpu.h"
*/
import "C"

import (
	"fmt"

	"github.com/hyperledger-labs/minbft/api"
)

// statusToErr maps an mbft_status to the reference's outcome: nil, a Go
// error with the reference's wording (authenticator.go:130-132 wraps the
// scheme error as "Invalid authentication tag"), or the panic of
// EcdsaSigCipher.Verify on malformed DER in an ECDSA role (crypto.go:82-84).
// Negative values are C-ABI failures (no GPU, out of memory): the
// reference cannot fail that way, so they panic rather than pass as a
// rejected message.
func statusToErr(role api.AuthenticationRole, st int) error {
	if st < 0 {
		panic(fmt.Sprintf("GPU authenticator failure: %d", st))
	}
	switch st {
	case C.MBFT_ACCEPT:
		return nil
	case C.MBFT_MALFORMED_DER:
		if role != api.USIGAuthen {
			panic("asn1: structure error") // crypto.go:82-84 panics on asn1.Unmarshal errors
		}
		return tagError("failed to unmarshal USIG signature") // usig-enclave.go:217-219
	case C.MBFT_REJECT_SIG:
		if role == api.USIGAuthen {
			return tagError("Failed to verify USIG certificate: invalid signature")
		}
		return tagError("Signature is not valid")
	case C.MBFT_DER_TRAILING:
		return tagError("extra bytes in USIG signature") // usig-enclave.go:220-221
	case C.MBFT_UNKNOWN_KEY:
		return tagError("public key not found")
	case C.MBFT_BAD_KEY:
		return tagError("invalid public key")
	case C.MBFT_BAD_UI:
		return tagError("failed to unmarshal UI") // usig/usig.go:75-80
	case C.MBFT_BAD_CERT:
		return tagError("failed to parse UI cert") // usig/sgx/sgx-usig.go:159-168
	case C.MBFT_EPOCH_MISMATCH:
		return tagError("Failed to verify USIG certificate: epoch value mismatch") // sgx-usig.go:92-94
	case C.MBFT_UNKNOWN_ROLE:
		return fmt.Errorf("Unknown role: %v", role) // authenticator.go:126-129, keymanager.go:100
	}
	return tagError(fmt.Sprintf("status %d", st))
}

func tagError(why string) error {
	return fmt.Errorf("Invalid authentication tag: %s", why)
}
