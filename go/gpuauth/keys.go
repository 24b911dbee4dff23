package gpuauth

// Which keys the GPU context holds.  The reference's authenticator verifies
// a call by ANY id its key store has a key for (SimpleKeyStore.NodePublicKey,
// sample/authentication/keymanager.go:96-101, over every key of keys.yaml,
// :179-227), so the binding must too:
//
//   - KeyIDsFromFile lists every id of every role in a keys.yaml (the file
//     LoadSimpleKeyStore reads), so a replica registers all of them at start
//     (sample/peer/cmd/gpu-stack.go), whatever their number or numbering;
//   - with Config.KeyStore set, a call whose (role, id) the context does not
//     hold yet is looked up in the store BEFORE its batch goes to the GPU
//     (ensureKeys) and, if the store has the key, registered first, at the
//     comb window of its role.  Registering before the batch -- not retrying
//     after an MBFT_UNKNOWN_KEY -- keeps every status, and the USIG epoch
//     state, exactly what the reference gives: the batch runs as if the key
//     had been there from the start.  An id the store does not have is
//     remembered as absent (the store is static) and rejected as the
//     reference rejects it (a nil key, crypto.go:85-88 / :192-195).

/*
#include "minbft_gpu.h"
*/
import "C"

import (
	"crypto/ecdsa"
	"fmt"
	"io"
	"io/ioutil"
	"sort"
	"sync"
	"unsafe"

	yaml "gopkg.in/yaml.v2"

	"github.com/hyperledger-labs/minbft/api"
)

// keyFile is the part of the reference's key store file the binding reads:
// the ids of each role's key set (keymanager.go:147-171 simpleKeyStoreFile,
// keySet, keyPair; the keys themselves come from the loaded store).
type keyFile struct {
	Replica *keyFileSet `yaml:"replica"`
	Usig    *keyFileSet `yaml:"usig"`
	Client  *keyFileSet `yaml:"client"`
}

type keyFileSet struct {
	Keys []keyFileEntry `yaml:"keys"`
}

type keyFileEntry struct {
	ID uint32 `yaml:"id"`
}

// KeyIDsFromFile returns, per role, the sorted ids that have a key in a
// keys.yaml.  A role whose key set is present has an entry even with no
// keys (the reference then knows the role: an unknown id is "invalid
// signature", not "key set not found", keymanager.go:96-101).
func KeyIDsFromFile(r io.Reader) (map[api.AuthenticationRole][]uint32, error) {
	b, err := ioutil.ReadAll(r)
	if err != nil {
		return nil, fmt.Errorf("read error: %v", err)
	}
	var f keyFile
	if err := yaml.Unmarshal(b, &f); err != nil {
		return nil, fmt.Errorf("yaml parse error: %v", err)
	}
	out := make(map[api.AuthenticationRole][]uint32)
	for role, set := range map[api.AuthenticationRole]*keyFileSet{
		api.ReplicaAuthen: f.Replica, api.USIGAuthen: f.Usig, api.ClientAuthen: f.Client} {
		if set == nil {
			continue
		}
		ids := make([]uint32, 0, len(set.Keys))
		for _, k := range set.Keys {
			ids = append(ids, k.ID)
		}
		sort.Slice(ids, func(i, j int) bool { return ids[i] < ids[j] })
		out[role] = ids
	}
	return out, nil
}

type roleID struct {
	role api.AuthenticationRole
	id   uint32
}

// maxAbsent bounds the remembered absent ids (a peer may send any id).
const maxAbsent = 1 << 16

// keyRegistry tracks the (role, id) pairs the context holds and the ones the
// key store does not have, and registers late keys.
type keyRegistry struct {
	mu      sync.RWMutex
	ks      PublicKeyStore
	windows Windows
	known   map[roleID]bool
	absent  map[roleID]bool
}

func (r *keyRegistry) init(ks PublicKeyStore, w Windows) {
	r.ks = ks
	r.windows = w
	r.known = make(map[roleID]bool)
	r.absent = make(map[roleID]bool)
}

func (r *keyRegistry) add(role api.AuthenticationRole, id uint32) {
	r.mu.Lock()
	r.known[roleID{role, id}] = true
	r.mu.Unlock()
}

func (r *keyRegistry) window(role api.AuthenticationRole) int {
	switch role {
	case api.ClientAuthen:
		return r.windows.Client
	case api.USIGAuthen:
		return r.windows.USIG
	}
	return r.windows.Replica
}

// ensure makes sure (role, id) is registered if the key store has a key for
// it.  Cheap when it is known or known absent (a read-locked map lookup).
func (a *Authenticator) ensureKey(role api.AuthenticationRole, id uint32) {
	r := &a.keys
	if r.ks == nil {
		return
	}
	if roleByte(role) == 0 {
		return // no scheme for the role: rejected as MBFT_UNKNOWN_ROLE whatever a key store holds
	}
	k := roleID{role, id}
	r.mu.RLock()
	done := r.known[k] || r.absent[k]
	r.mu.RUnlock()
	if done {
		return
	}
	r.mu.Lock()
	defer r.mu.Unlock()
	if r.known[k] || r.absent[k] {
		return
	}
	miss := func() {
		if len(r.absent) >= maxAbsent {
			r.absent = make(map[roleID]bool)
		}
		r.absent[k] = true
	}
	pk, err := r.ks.NodePublicKey(role, id)
	if err != nil || pk == nil {
		miss() // no key set for the role, or no key for the id: the reference rejects
		return
	}
	epk, ok := pk.(*ecdsa.PublicKey)
	if !ok {
		miss()
		return
	}
	xy, err := rawXY(epk)
	if err != nil {
		miss()
		return
	}
	// the context-wide "window for keys registered next": set under r.mu,
	// the only place keys are added after New
	if C.mbft_set_key_window(a.ctx, C.int(r.window(role))) != C.MBFT_OK {
		return // left unknown: the call is rejected as with no key, retried next time
	}
	C.mbft_add_role(a.ctx, C.uint32_t(role))
	if C.mbft_set_public_key_xy(a.ctx, C.uint32_t(role), C.uint32_t(id),
		(*C.uint8_t)(unsafe.Pointer(&xy[0]))) != C.MBFT_OK {
		return
	}
	r.known[k] = true
}

// ensureKeys runs ensureKey over the signers of a batch (consecutive calls
// by the same signer are looked up once).
func (a *Authenticator) ensureKeys(calls []Call) {
	if a.keys.ks == nil {
		return
	}
	var last roleID
	for i, c := range calls {
		k := roleID{c.Role, c.ID}
		if i > 0 && k == last {
			continue
		}
		last = k
		a.ensureKey(c.Role, c.ID)
	}
}
