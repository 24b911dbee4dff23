package gpuauth

// Restates the reference's own authentication tests through the GPU
// authenticator, with the reference's fixture key pair
// (sample/authentication/keymanager_test.go:68-69).  Needs an MI355X and
// the built library; the same scenarios run in Python through the C-ABI in
// tests/test_reference_scenarios.py.

import (
	"crypto/ecdsa"
	"crypto/elliptic"
	"crypto/rand"
	"crypto/sha256"
	"crypto/x509"
	"encoding/base64"
	"encoding/binary"
	"fmt"
	"reflect"
	"strings"
	"sync"
	"testing"

	"github.com/hyperledger-labs/minbft/api"
)

const fixturePriv = "MHcCAQEEIFxopskcl2LyZ/LLsDMBfQk/82WZQI/YhvXNSYZNmUSFoAoGCCqGSM49AwEHoUQDQgAEh6uiVdr+3EgyT3YEilvrvzQINr8eolxR22/0JudQrpGbLQQQIK+7RdnoLaIyZIlakZkb1tAws0iQN263EkwzGw=="

func fixtureKey(t *testing.T) *ecdsa.PrivateKey {
	der, err := base64.StdEncoding.DecodeString(fixturePriv)
	if err != nil {
		t.Fatal(err)
	}
	sk, err := x509.ParseECPrivateKey(der)
	if err != nil {
		t.Fatal(err)
	}
	return sk
}

func newTestAuth(t *testing.T) *Authenticator {
	sk := fixtureKey(t)
	keys := map[api.AuthenticationRole]map[uint32]*ecdsa.PublicKey{
		api.ReplicaAuthen: {0: &sk.PublicKey, 1: &sk.PublicKey, 2: &sk.PublicKey},
		api.ClientAuthen:  {10: &sk.PublicKey},
	}
	a, err := New(keys, false, Config{GeneratorWindow: 16, ReplicaWindow: 16, ClientWindow: 16,
		PrivateKeys: map[api.AuthenticationRole]*ecdsa.PrivateKey{
			api.ReplicaAuthen: sk, api.ClientAuthen: sk}})
	if err != nil {
		t.Fatal(err)
	}
	return a
}

// crypto_test.go:60-68, authenticator_test.go:29-69: generate, then verify.
func TestRoundTrip(t *testing.T) {
	a := newTestAuth(t)
	defer a.Close()
	msg := []byte("hello")
	for _, role := range []api.AuthenticationRole{api.ReplicaAuthen, api.ClientAuthen} {
		tag, err := a.GenerateMessageAuthenTag(role, msg)
		if err != nil {
			t.Fatal(err)
		}
		id := uint32(0)
		if role == api.ClientAuthen {
			id = 10
		}
		if err := a.VerifyMessageAuthenTag(role, id, msg, tag); err != nil {
			t.Errorf("role %v: %v", role, err)
		}
		if err := a.VerifyMessageAuthenTag(role, id, []byte("hellp"), tag); err == nil {
			t.Errorf("role %v: tampered message accepted", role)
		}
	}
}

// VerifyBatch gives the single-call results.
func TestBatchForms(t *testing.T) {
	a := newTestAuth(t)
	defer a.Close()
	var calls []Call
	for i := 0; i < 1000; i++ {
		msg := []byte{byte(i), byte(i >> 8), 'x'}
		tag, err := a.GenerateMessageAuthenTag(api.ReplicaAuthen, msg)
		if err != nil {
			t.Fatal(err)
		}
		if i%7 == 0 {
			msg = append([]byte{}, msg...)
			msg[0] ^= 1
		}
		calls = append(calls, Call{Role: api.ReplicaAuthen, ID: uint32(i % 3), Msg: msg, Tag: tag})
	}
	errs := a.VerifyBatch(calls)
	for i, c := range calls {
		single := a.VerifyMessageAuthenTag(c.Role, c.ID, c.Msg, c.Tag)
		if (errs[i] == nil) != (single == nil) || (errs[i] == nil) != (i%7 != 0) {
			t.Fatalf("call %d: batch %v, single %v", i, errs[i], single)
		}
	}
}

// Concurrent VerifyBatch / VerifyMessageAuthenTag from many
// goroutines (api/api.go:132: methods may be invoked from spawned
// goroutines) give the single-call results; the library overlaps the
// batches (Config.Concurrency).
func TestConcurrentBatches(t *testing.T) {
	a := newTestAuth(t)
	defer a.Close()
	const streams, per = 8, 300
	all := make([][]Call, streams)
	for g := 0; g < streams; g++ {
		for i := 0; i < per; i++ {
			msg := []byte{byte(g), byte(i), byte(i >> 8), 'y'}
			tag, err := a.GenerateMessageAuthenTag(api.ReplicaAuthen, msg)
			if err != nil {
				t.Fatal(err)
			}
			if i%5 == 0 {
				msg = append([]byte{}, msg...)
				msg[1] ^= 0x80
			}
			all[g] = append(all[g], Call{Role: api.ReplicaAuthen, ID: uint32(i % 3), Msg: msg, Tag: tag})
		}
	}
	var wg sync.WaitGroup
	errc := make(chan string, streams)
	for g := 0; g < streams; g++ {
		wg.Add(1)
		go func(calls []Call) {
			defer wg.Done()
			errs := a.VerifyBatch(calls)
			for i, c := range calls {
				single := a.VerifyMessageAuthenTag(c.Role, c.ID, c.Msg, c.Tag)
				if (errs[i] == nil) != (single == nil) || (errs[i] == nil) != (i%5 != 0) {
					errc <- "mismatch"
					return
				}
			}
		}(all[g])
	}
	wg.Wait()
	close(errc)
	for e := range errc {
		t.Fatal(e)
	}
}

// KeyIDsFromFile lists every id of every key set of a keys.yaml in the
// reference's layout (keymanager.go:125-171), non-contiguous ids included
// (no GPU needed).
func TestKeyIDsFromFile(t *testing.T) {
	const y = `
replica:
  keyspec: ECDSA
  keys:
    - {id: 2, privateKey: a, publicKey: b}
    - {id: 0, privateKey: a, publicKey: b}
    - {id: 1, privateKey: a, publicKey: b}
usig:
  keyspec: SGX_ECDSA
  keys:
    - {id: 0, privateKey: a, publicKey: b}
client:
  keyspec: ECDSA
  keys: []
`
	ids, err := KeyIDsFromFile(strings.NewReader(y))
	if err != nil {
		t.Fatal(err)
	}
	want := map[api.AuthenticationRole][]uint32{
		api.ReplicaAuthen: {0, 1, 2}, api.USIGAuthen: {0}, api.ClientAuthen: {}}
	if !reflect.DeepEqual(ids, want) {
		t.Fatalf("got %v, want %v", ids, want)
	}
	ids, err = KeyIDsFromFile(strings.NewReader("replica:\n  keys:\n    - {id: 7}\n"))
	if err != nil || len(ids) != 1 || !reflect.DeepEqual(ids[api.ReplicaAuthen], []uint32{7}) {
		t.Fatalf("got %v %v", ids, err)
	}
}

// mapStore is a key store with the reference's NodePublicKey contract
// (keymanager.go:96-101): an error for a role without a key set, a nil key
// for an unknown id.
type mapStore map[api.AuthenticationRole]map[uint32]*ecdsa.PublicKey

func (m mapStore) NodePublicKey(role api.AuthenticationRole, id uint32) (interface{}, error) {
	keys, ok := m[role]
	if !ok {
		return nil, fmt.Errorf("key set not found for role=%v, id=%d", role, id)
	}
	if k, ok := keys[id]; ok {
		return k, nil
	}
	return nil, nil
}

// Several clients with non-contiguous ids: every id the store holds is
// verified -- the ones given to New and, through Config.KeyStore, the ones
// registered on first use -- and an id the store lacks is rejected as the
// reference rejects it ("invalid signature": a nil key, crypto.go:85-88).
func TestClientsNotGivenToNew(t *testing.T) {
	sk := fixtureKey(t)
	other, err := ecdsa.GenerateKey(elliptic.P256(), rand.Reader)
	if err != nil {
		t.Fatal(err)
	}
	store := mapStore{
		api.ReplicaAuthen: {0: &sk.PublicKey},
		api.ClientAuthen:  {3: &sk.PublicKey, 17: &other.PublicKey, 4096: &sk.PublicKey},
	}
	ids := map[api.AuthenticationRole][]uint32{api.ReplicaAuthen: {0}, api.ClientAuthen: {3}}
	keys, err := KeysFromStore(store, ids)
	if err != nil {
		t.Fatal(err)
	}
	a, err := New(keys, false, Config{GeneratorWindow: 16, ReplicaWindow: 16, ClientWindow: 8,
		KeyStore: store, PrivateKeys: map[api.AuthenticationRole]*ecdsa.PrivateKey{api.ClientAuthen: sk}})
	if err != nil {
		t.Fatal(err)
	}
	defer a.Close()
	msg := []byte("REQUEST from a client")
	tag, err := a.GenerateMessageAuthenTag(api.ClientAuthen, msg)
	if err != nil {
		t.Fatal(err)
	}
	otherTag, err := ecdsaScheme.GenerateAuthenticationTag(msg, other)
	if err != nil {
		t.Fatal(err)
	}
	calls := []Call{
		{Role: api.ClientAuthen, ID: 3, Msg: msg, Tag: tag},
		{Role: api.ClientAuthen, ID: 4096, Msg: msg, Tag: tag},     // not given to New
		{Role: api.ClientAuthen, ID: 17, Msg: msg, Tag: otherTag},  // not given to New
		{Role: api.ClientAuthen, ID: 99, Msg: msg, Tag: tag},       // not in the store
		{Role: api.ClientAuthen, ID: 17, Msg: msg, Tag: tag},       // wrong signer
	}
	want := []bool{true, true, true, false, false}
	for i, err := range a.VerifyBatch(calls) {
		if (err == nil) != want[i] {
			t.Fatalf("batch call %d: %v", i, err)
		}
	}
	for i, c := range calls {
		if err := a.VerifyMessageAuthenTag(c.Role, c.ID, c.Msg, c.Tag); (err == nil) != want[i] {
			t.Fatalf("call %d: %v", i, err)
		}
	}
}

// requestAuthenBytes is messages.AuthenBytes of a REQUEST
// (messages/authen.go:33,54-56), to sign test requests.
func requestAuthenBytes(seq uint64, op []byte) []byte {
	h := sha256.Sum256(op)
	b := append([]byte("REQUEST"), make([]byte, 8)...)
	binary.BigEndian.PutUint64(b[7:], seq)
	return append(b, h[:]...)
}

// CheckMessages + Resolve in order give the reference validator's outcome
// per REQUEST (the client stream's validator, core/request.go:146-150):
// nil, "invalid signature", and the panic on a malformed DER signature.
func TestCheckMessagesRequests(t *testing.T) {
	a := newTestAuth(t)
	defer a.Close()
	sk := fixtureKey(t)
	var msgs []api.AuthenMessage
	for i := 0; i < 300; i++ {
		op := []byte{byte(i), byte(i >> 8), 'o', 'p'}
		tag, err := ecdsaScheme.GenerateAuthenticationTag(requestAuthenBytes(uint64(i+1), op), sk)
		if err != nil {
			t.Fatal(err)
		}
		if i%10 == 3 {
			op = append([]byte{}, op...)
			op[0] ^= 1 // tampered operation: SHA256(op) changes inside e
		}
		msgs = append(msgs, api.AuthenMessage{Type: api.AuthenRequest, ClientID: 10,
			Seq: uint64(i + 1), Op: op, Sig: tag})
	}
	msgs = append(msgs, api.AuthenMessage{Type: api.AuthenRequest, ClientID: 10, Seq: 9,
		Op: []byte("x"), Sig: []byte{0x31, 0x00}})
	b, err := a.CheckMessages(msgs, 3)
	if err != nil {
		t.Fatal(err)
	}
	defer b.Close()
	for i := 0; i < 300; i++ {
		if err := b.Resolve(i); (err == nil) != (i%10 != 3) {
			t.Fatalf("message %d: %v", i, err)
		}
	}
	defer func() {
		if recover() == nil {
			t.Fatal("malformed DER did not panic")
		}
	}()
	_ = b.Resolve(300)
}
