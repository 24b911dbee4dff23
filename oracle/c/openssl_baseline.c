/*
 * CPU baseline ("not Go"), TEST/BENCH INFRASTRUCTURE ONLY: the reference's
 * per-call ECDSA-role work -- VerifyMessageAuthenTag in
 * sample/authentication/crypto.go:79-89,120-126: DER-decode the tag
 * (asn1.Unmarshal at crypto.go:81), digest = msg || SHA256("") (the Sum(m)
 * quirk at crypto.go:121, so e = the first 32 bytes), ecdsa.Verify
 * (crypto.go:86) -- over OpenSSL 3's d2i_ECDSA_SIG + ECDSA_do_verify,
 * one pthread per core.  Used only by bench.py's cpu_baseline leg; never
 * by the product.  OpenSSL's P-256 verify is an independent, heavily
 * optimized implementation of the same arithmetic as Go's crypto/ecdsa
 * (the Go toolchain is absent from this image and the GPU box).
 */
#define OPENSSL_SUPPRESS_DEPRECATED
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static const uint8_t kEmptyHash[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14,
                                       0x9a, 0xfb, 0xf4, 0xc8, 0x99, 0x6f, 0xb9, 0x24,
                                       0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b, 0x93, 0x4c,
                                       0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};

typedef struct {
  const uint8_t *qxy;                 /* nkeys x 64 B (X || Y big-endian) */
  size_t nkeys;
  const uint32_t *slot;
  const uint8_t *msgs, *tags;
  const uint64_t *moff, *toff;
  size_t lo, hi;
  uint8_t *out;                       /* 0 accept, 1 reject, 2 malformed DER */
  int rc;
} job;

static EC_KEY *make_key(const uint8_t *xy) {
  EC_KEY *k = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
  BIGNUM *x = BN_bin2bn(xy, 32, NULL), *y = BN_bin2bn(xy + 32, 32, NULL);
  int ok = k && x && y && EC_KEY_set_public_key_affine_coordinates(k, x, y) == 1;
  BN_free(x);
  BN_free(y);
  if (!ok) {
    EC_KEY_free(k);
    return NULL;
  }
  return k;
}

static void *run(void *p) {
  job *j = (job *)p;
  EC_KEY **keys = calloc(j->nkeys, sizeof(EC_KEY *));
  if (!keys) {
    j->rc = -1;
    return NULL;
  }
  for (size_t k = 0; k < j->nkeys; k++) keys[k] = make_key(j->qxy + 64 * k);
  for (size_t i = j->lo; i < j->hi; i++) {
    const uint8_t *m = j->msgs + j->moff[i];
    const size_t ml = j->moff[i + 1] - j->moff[i];
    const uint8_t *t = j->tags + j->toff[i];
    const long tl = (long)(j->toff[i + 1] - j->toff[i]);
    ECDSA_SIG *sig = d2i_ECDSA_SIG(NULL, &t, tl);
    if (!sig) {
      j->out[i] = 2;
      continue;
    }
    uint8_t e[32];
    for (size_t k = 0; k < 32; k++) e[k] = k < ml ? m[k] : kEmptyHash[k - ml];
    const uint32_t s = j->slot[i];
    const int ok = s < j->nkeys && keys[s] && ECDSA_do_verify(e, 32, sig, keys[s]) == 1;
    j->out[i] = ok ? 0 : 1;
    ECDSA_SIG_free(sig);
  }
  for (size_t k = 0; k < j->nkeys; k++) EC_KEY_free(keys[k]);
  free(keys);
  j->rc = 0;
  return NULL;
}

int ossl_verify_ecdsa_role_batch(const uint8_t *qxy, size_t nkeys, const uint32_t *slot,
                                 const uint8_t *msgs, const uint64_t *moff, const uint8_t *tags,
                                 const uint64_t *toff, size_t n, uint8_t *out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  job *jobs = calloc((size_t)nthreads, sizeof(job));
  if (!th || !jobs) return -1;
  for (int t = 0; t < nthreads; t++) {
    job *j = &jobs[t];
    j->qxy = qxy;
    j->nkeys = nkeys;
    j->slot = slot;
    j->msgs = msgs;
    j->tags = tags;
    j->moff = moff;
    j->toff = toff;
    j->lo = n * (size_t)t / (size_t)nthreads;
    j->hi = n * (size_t)(t + 1) / (size_t)nthreads;
    j->out = out;
    pthread_create(&th[t], NULL, run, j);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  free(th);
  free(jobs);
  return rc;
}
