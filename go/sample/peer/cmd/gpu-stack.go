// GPU authenticator for the sample replica (a new file for package cmd of
// sample/peer/cmd, next to run.go).  Not built in this image (no Go
// toolchain); INTEGRATION.md §2 shows the two-line change to run.go that
// uses it.  Go 1.11 compatible (go.mod:30).

package cmd

import (
	"fmt"
	"io"
	"os"

	"github.com/hyperledger-labs/minbft/api"
	authen "github.com/hyperledger-labs/minbft/sample/authentication"
	"github.com/hyperledger-labs/minbft/sample/authentication/gpuauth"
)

// gpuReplicaStack is replicaStack (run.go) with the GPU authenticator:
// embedding *gpuauth.Authenticator also promotes its CheckMessages, so
// minbft.New finds an api.MessageBatchChecker and installs the batched
// stream loop (core/message-handling-batch.go).
type gpuReplicaStack struct {
	api.ReplicaConnector
	*gpuauth.Authenticator
	api.RequestConsumer
}

// newGPUAuthenticator builds the GPU authenticator over EVERY public key of
// keys.yaml (the file authen.NewWithSGXUSIG reads): all ids of each role's
// key set, however many and however numbered, as LoadSimpleKeyStore loads
// them (sample/authentication/keymanager.go:179-227) -- the reference
// verifies any id present there (keymanager.go:96-101).  The loaded store
// also backs late registration (gpuauth.Config.KeyStore).  Generation (the
// replica's own signatures and USIG UIs) stays with sgxAuth, the reference
// authenticator.
func newGPUAuthenticator(keysPath string, id uint32, sgxAuth api.Authenticator) (*gpuauth.Authenticator, error) {
	f, err := os.Open(keysPath)
	if err != nil {
		return nil, fmt.Errorf("Failed to open keyset file: %s", err)
	}
	defer f.Close()
	ids, err := gpuauth.KeyIDsFromFile(f)
	if err != nil {
		return nil, fmt.Errorf("failed to read key ids: %v", err)
	}
	if _, err := f.Seek(0, io.SeekStart); err != nil {
		return nil, err
	}
	ks, err := authen.LoadSimpleKeyStore(f, []api.AuthenticationRole{api.ReplicaAuthen, api.USIGAuthen}, id)
	if err != nil {
		return nil, fmt.Errorf("failed to load keystore: %v", err)
	}
	keys, err := gpuauth.KeysFromStore(ks, ids)
	if err != nil {
		return nil, err
	}
	return gpuauth.New(keys, true, gpuauth.Config{Generator: sgxAuth, KeyStore: ks})
}
