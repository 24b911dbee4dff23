// GPU authenticator for the sample replica (a new file for package cmd of
// sample/peer/cmd, next to run.go).  Not built in this image (no Go
// toolchain); INTEGRATION.md §2 shows the two-line change to run.go that
// uses it.  Go 1.11 compatible (go.mod:30).

package cmd

import (
	"fmt"
	"os"

	"github.com/hyperledger-labs/minbft/api"
	authen "github.com/hyperledger-labs/minbft/sample/authentication"
	"github.com/hyperledger-labs/minbft/sample/authentication/gpuauth"
)

// gpuReplicaStack is replicaStack (run.go) with the GPU authenticator:
// embedding *gpuauth.Authenticator also promotes its Prefetch, so
// minbft.New finds an api.AuthenPrefetcher and installs the batched stream
// loop (core/message-handling-batch.go).
type gpuReplicaStack struct {
	api.ReplicaConnector
	*gpuauth.Authenticator
	api.RequestConsumer
}

// newGPUAuthenticator builds the GPU authenticator over the public keys of
// keys.yaml (the file authen.NewWithSGXUSIG reads): replicas and USIG
// instances 0..n-1, clients 0..nClients-1.  Generation (the replica's own
// signatures and USIG UIs) stays with sgxAuth, the reference authenticator.
func newGPUAuthenticator(keysPath string, id, n, nClients uint32,
	sgxAuth api.Authenticator) (*gpuauth.Authenticator, error) {
	f, err := os.Open(keysPath)
	if err != nil {
		return nil, fmt.Errorf("Failed to open keyset file: %s", err)
	}
	defer f.Close()
	ks, err := authen.LoadSimpleKeyStore(f, []api.AuthenticationRole{api.ReplicaAuthen, api.USIGAuthen}, id)
	if err != nil {
		return nil, fmt.Errorf("failed to load keystore: %v", err)
	}
	ids := map[api.AuthenticationRole][]uint32{}
	for i := uint32(0); i < n; i++ {
		ids[api.ReplicaAuthen] = append(ids[api.ReplicaAuthen], i)
		ids[api.USIGAuthen] = append(ids[api.USIGAuthen], i)
	}
	for i := uint32(0); i < nClients; i++ {
		ids[api.ClientAuthen] = append(ids[api.ClientAuthen], i)
	}
	keys, err := gpuauth.KeysFromStore(ks, ids)
	if err != nil {
		return nil, err
	}
	return gpuauth.New(keys, true, gpuauth.Config{Generator: sgxAuth})
}
