/*
 * p256_oracle.c -- C restatement of MinBFT's message-authentication checks.
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/ (bulk parity of the GPU path at
 * sizes the Python oracle cannot reach), __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.  The product (minbft_amd/) never links it.
 *
 * Restates, independently of the GPU implementation (different algorithm:
 * 4x64-bit Montgomery, 4-bit windowed Straus-Shamir with complete Jacobian
 * additions, its own SHA-256 and DER decoder):
 *   - Go crypto/ecdsa.Verify (Go 1.11/1.14, pinned by go.mod:30 and
 *     .github/workflows/continuous-integration.yml:15): r,s in [1, N-1],
 *     e = hashToInt(left-most 32 bytes), w = s^-1, u1 = e w, u2 = r w,
 *     (x, y) = u1 G + u2 Q, infinity -> false, accept iff x mod N == r.
 *   - encoding/asn1 decode of struct{R, S *big.Int} (crypto.go:81,
 *     usig-enclave.go:217), following oracle/p256.py's restatement.
 *   - the digests: quirk md = m || SHA256("") (crypto.go:114,121) and the USIG
 *     chain SHA256(SHA256(m) || epoch_le || ctr_le) (usig-enclave.go:204-214).
 * Pinned against oracle/p256.py and OpenSSL by tests/test_oracle.py.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } u256;

/* ------------------------------------------------------------ constants */
static const u256 P = {{0xFFFFFFFFFFFFFFFFull, 0x00000000FFFFFFFFull, 0x0000000000000000ull,
                        0xFFFFFFFF00000001ull}};
static const u256 N = {{0xF3B9CAC2FC632551ull, 0xBCE6FAADA7179E84ull, 0xFFFFFFFFFFFFFFFFull,
                        0xFFFFFFFF00000000ull}};
static const u256 B = {{0x3BCE3C3E27D2604Bull, 0x651D06B0CC53B0F6ull, 0xB3EBBD55769886BCull,
                        0x5AC635D8AA3A93E7ull}};
static const u256 GX = {{0xF4A13945D898C296ull, 0x77037D812DEB33A0ull, 0xF8BCE6E563A440F2ull,
                         0x6B17D1F2E12C4247ull}};
static const u256 GY = {{0xCBB6406837BF51F5ull, 0x2BCE33576B315ECEull, 0x8EE7EB4A7C0F9E16ull,
                         0x4FE342E2FE1A7F9Bull}};

typedef struct {
  u256 m;      /* modulus */
  uint64_t n0; /* -m^-1 mod 2^64 */
  u256 r2;     /* 2^512 mod m */
  u256 one;    /* 2^256 mod m */
} modctx;

static modctx MP, MN;

/* ------------------------------------------------------------- u256 ops */
static int u256_cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; i--) {
    if (a->v[i] < b->v[i]) return -1;
    if (a->v[i] > b->v[i]) return 1;
  }
  return 0;
}
static int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static uint64_t u256_add(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
static uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a->v[i] - b->v[i] - borrow;
    r->v[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
  return borrow;
}
static void u256_from_be(u256* r, const uint8_t* be) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) w = (w << 8) | be[8 * (3 - i) + j];
    r->v[i] = w;
  }
}
static int u256_bit(const u256* a, int i) { return (int)((a->v[i >> 6] >> (i & 63)) & 1); }

/* --------------------------------------------------- modular arithmetic */
static void mod_add(const modctx* M, u256* r, const u256* a, const u256* b) {
  u256 t;
  uint64_t c = u256_add(&t, a, b);
  u256 d;
  uint64_t br = u256_sub(&d, &t, &M->m);
  *r = (c || !br) ? d : t;
}
static void mod_sub(const modctx* M, u256* r, const u256* a, const u256* b) {
  u256 t;
  uint64_t br = u256_sub(&t, a, b);
  if (br) u256_add(&t, &t, &M->m);
  *r = t;
}
/* Montgomery CIOS: r = a b 2^-256 mod m */
static void mont_mul(const modctx* M, u256* r, const u256* a, const u256* b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * M->n0;
    c = (u128)m * M->m.v[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * M->m.v[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  u256 d;
  uint64_t br = u256_sub(&d, &res, &M->m);
  *r = (t[4] || !br) ? d : res;
}
static void to_mont(const modctx* M, u256* r, const u256* a) { mont_mul(M, r, a, &M->r2); }
static void from_mont(const modctx* M, u256* r, const u256* a) {
  u256 one = {{1, 0, 0, 0}};
  mont_mul(M, r, a, &one);
}
/* a^(m-2) in the Montgomery domain */
static void mod_inv(const modctx* M, u256* r, const u256* a) {
  u256 e, two = {{2, 0, 0, 0}};
  u256_sub(&e, &M->m, &two);
  u256 acc = M->one;
  for (int i = 255; i >= 0; i--) {
    mont_mul(M, &acc, &acc, &acc);
    if (u256_bit(&e, i)) mont_mul(M, &acc, &acc, a);
  }
  *r = acc;
}

static void modctx_init(modctx* M, const u256* m) {
  M->m = *m;
  /* n0 = -m^-1 mod 2^64 by Newton iteration */
  uint64_t inv = 1;
  for (int i = 0; i < 7; i++) inv *= 2 - m->v[0] * inv;
  M->n0 = (uint64_t)0 - inv;
  /* one = 2^256 mod m = (2^256 - m) since m > 2^255 */
  u256 zero = {{0, 0, 0, 0}};
  u256_sub(&M->one, &zero, m);
  /* r2 = 2^512 mod m by 256 modular doublings of one */
  u256 x = M->one;
  for (int i = 0; i < 256; i++) mod_add(M, &x, &x, &x);
  M->r2 = x;
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_once(void) {
  modctx_init(&MP, &P);
  modctx_init(&MN, &N);
}

/* -------------------------------------------------------------- points */
typedef struct { u256 X, Y, Z; int inf; } jpt; /* Montgomery-form coords */

static void pt_dbl(jpt* r, const jpt* a) {
  if (a->inf) { *r = *a; return; }
  const modctx* M = &MP;
  u256 delta, gamma, beta, t1, t2, alpha, t;
  mont_mul(M, &delta, &a->Z, &a->Z);
  mont_mul(M, &gamma, &a->Y, &a->Y);
  mont_mul(M, &beta, &a->X, &gamma);
  mod_sub(M, &t1, &a->X, &delta);
  mod_add(M, &t2, &a->X, &delta);
  mont_mul(M, &alpha, &t1, &t2);
  mod_add(M, &t, &alpha, &alpha);
  mod_add(M, &alpha, &t, &alpha); /* 3(X-d)(X+d) */
  jpt o;
  o.inf = 0;
  mod_add(M, &t, &a->Y, &a->Z);
  mont_mul(M, &t, &t, &t);
  mod_sub(M, &t, &t, &gamma);
  mod_sub(M, &o.Z, &t, &delta);
  u256 b4, b8;
  mod_add(M, &b4, &beta, &beta);
  mod_add(M, &b4, &b4, &b4);
  mod_add(M, &b8, &b4, &b4);
  mont_mul(M, &t, &alpha, &alpha);
  mod_sub(M, &o.X, &t, &b8);
  mod_sub(M, &t, &b4, &o.X);
  mont_mul(M, &t, &t, &alpha);
  u256 g2;
  mont_mul(M, &g2, &gamma, &gamma);
  mod_add(M, &g2, &g2, &g2);
  mod_add(M, &g2, &g2, &g2);
  mod_add(M, &g2, &g2, &g2);
  mod_sub(M, &o.Y, &t, &g2);
  *r = o;
}

/* complete Jacobian addition (add-2007-bl with special cases) */
static void pt_add(jpt* r, const jpt* a, const jpt* b) {
  if (a->inf) { *r = *b; return; }
  if (b->inf) { *r = *a; return; }
  const modctx* M = &MP;
  u256 z1z1, z2z2, u1, u2, s1, s2, t;
  mont_mul(M, &z1z1, &a->Z, &a->Z);
  mont_mul(M, &z2z2, &b->Z, &b->Z);
  mont_mul(M, &u1, &a->X, &z2z2);
  mont_mul(M, &u2, &b->X, &z1z1);
  mont_mul(M, &t, &b->Z, &z2z2);
  mont_mul(M, &s1, &a->Y, &t);
  mont_mul(M, &t, &a->Z, &z1z1);
  mont_mul(M, &s2, &b->Y, &t);
  if (u256_cmp(&u1, &u2) == 0) {
    if (u256_cmp(&s1, &s2) == 0) { pt_dbl(r, a); return; }
    r->inf = 1;
    return;
  }
  u256 h, i, j, rr, v;
  mod_sub(M, &h, &u2, &u1);
  mod_add(M, &i, &h, &h);
  mont_mul(M, &i, &i, &i);
  mont_mul(M, &j, &h, &i);
  mod_sub(M, &rr, &s2, &s1);
  mod_add(M, &rr, &rr, &rr);
  mont_mul(M, &v, &u1, &i);
  jpt o;
  o.inf = 0;
  mont_mul(M, &t, &rr, &rr);
  mod_sub(M, &t, &t, &j);
  mod_sub(M, &t, &t, &v);
  mod_sub(M, &o.X, &t, &v);
  mod_sub(M, &t, &v, &o.X);
  mont_mul(M, &t, &t, &rr);
  u256 s1j;
  mont_mul(M, &s1j, &s1, &j);
  mod_add(M, &s1j, &s1j, &s1j);
  mod_sub(M, &o.Y, &t, &s1j);
  mod_add(M, &t, &a->Z, &b->Z);
  mont_mul(M, &t, &t, &t);
  mod_sub(M, &t, &t, &z1z1);
  mod_sub(M, &t, &t, &z2z2);
  mont_mul(M, &o.Z, &t, &h);
  *r = o;
}

static int on_curve_plain(const u256* x, const u256* y) {
  if (u256_cmp(x, &P) >= 0 || u256_cmp(y, &P) >= 0) return 0;
  const modctx* M = &MP;
  u256 xm, ym, bm, l, rgt, t;
  to_mont(M, &xm, x);
  to_mont(M, &ym, y);
  to_mont(M, &bm, &B);
  mont_mul(M, &l, &ym, &ym);
  mont_mul(M, &t, &xm, &xm);
  mont_mul(M, &rgt, &t, &xm);
  mod_sub(M, &rgt, &rgt, &xm);
  mod_sub(M, &rgt, &rgt, &xm);
  mod_sub(M, &rgt, &rgt, &xm);
  mod_add(M, &rgt, &rgt, &bm);
  return u256_cmp(&l, &rgt) == 0;
}

/* -------------------------------------------------- crypto/ecdsa.Verify */
/* e32: left-most 32 bytes of the digest (big-endian); r32/s32 big-endian
 * values (callers map non-positive or >= 2^256 DER integers to zero).
 * Returns 1 = accept, 0 = reject, -1 = invalid key (off-curve). */
int oracle_ecdsa_verify(const uint8_t qxy[64], const uint8_t e32[32], const uint8_t r32[32],
                        const uint8_t s32[32]) {
  pthread_once(&g_once, init_once);
  u256 qx, qy, e, r, s;
  u256_from_be(&qx, qxy);
  u256_from_be(&qy, qxy + 32);
  if (!on_curve_plain(&qx, &qy)) return -1;
  u256_from_be(&e, e32);
  u256_from_be(&r, r32);
  u256_from_be(&s, s32);
  if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
  if (u256_cmp(&r, &N) >= 0 || u256_cmp(&s, &N) >= 0) return 0;
  /* w = s^-1; u1 = e w; u2 = r w   (mod N) */
  u256 sm, w, em, rm, u1m, u2m, u1, u2;
  to_mont(&MN, &sm, &s);
  mod_inv(&MN, &w, &sm);
  /* e may be >= N: reduce once (e < 2^256 < 2N) */
  if (u256_cmp(&e, &N) >= 0) u256_sub(&e, &e, &N);
  to_mont(&MN, &em, &e);
  to_mont(&MN, &rm, &r);
  mont_mul(&MN, &u1m, &em, &w);
  mont_mul(&MN, &u2m, &rm, &w);
  from_mont(&MN, &u1, &u1m);
  from_mont(&MN, &u2, &u2m);
  /* tables k*G, k*Q for k = 0..15 */
  jpt TG[16], TQ[16];
  TG[0].inf = TQ[0].inf = 1;
  TG[1].inf = TQ[1].inf = 0;
  to_mont(&MP, &TG[1].X, &GX);
  to_mont(&MP, &TG[1].Y, &GY);
  TG[1].Z = MP.one;
  to_mont(&MP, &TQ[1].X, &qx);
  to_mont(&MP, &TQ[1].Y, &qy);
  TQ[1].Z = MP.one;
  for (int k = 2; k < 16; k++) {
    pt_add(&TG[k], &TG[k - 1], &TG[1]);
    pt_add(&TQ[k], &TQ[k - 1], &TQ[1]);
  }
  jpt acc;
  acc.inf = 1;
  for (int nib = 63; nib >= 0; nib--) {
    for (int d = 0; d < 4; d++) pt_dbl(&acc, &acc);
    const int a = (int)((u1.v[nib >> 4] >> (4 * (nib & 15))) & 15);
    const int b = (int)((u2.v[nib >> 4] >> (4 * (nib & 15))) & 15);
    if (a) pt_add(&acc, &acc, &TG[a]);
    if (b) pt_add(&acc, &acc, &TQ[b]);
  }
  if (acc.inf) return 0;
  u256 zi, zi2, x;
  mod_inv(&MP, &zi, &acc.Z);
  mont_mul(&MP, &zi2, &zi, &zi);
  mont_mul(&MP, &x, &acc.X, &zi2);
  from_mont(&MP, &x, &x);
  if (u256_cmp(&x, &N) >= 0) u256_sub(&x, &x, &N);
  return u256_cmp(&x, &r) == 0;
}

/* --------------------------------------------------------------- SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
    0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
    0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
    0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
    0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
    0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
    0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
    0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(uint32_t h[8], const uint8_t* p) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
           ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
void oracle_sha256(const uint8_t* m, size_t n, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= n; i += 64) sha_block(h, m + i);
  uint8_t buf[128];
  size_t rem = n - i;
  memcpy(buf, m + i, rem);
  buf[rem] = 0x80;
  size_t tot = rem + 1 + 8 <= 64 ? 64 : 128;
  memset(buf + rem + 1, 0, tot - rem - 1);
  uint64_t bits = (uint64_t)n * 8;
  for (int k = 0; k < 8; k++) buf[tot - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha_block(h, buf);
  if (tot == 128) sha_block(h, buf + 64);
  for (int k = 0; k < 8; k++) {
    out[4 * k] = (uint8_t)(h[k] >> 24);
    out[4 * k + 1] = (uint8_t)(h[k] >> 16);
    out[4 * k + 2] = (uint8_t)(h[k] >> 8);
    out[4 * k + 3] = (uint8_t)h[k];
  }
}

/* ------------------------------------------------ encoding/asn1 (Go rules) */
/* returns 1 ok, 0 error; follows oracle/p256.py _parse_tag_and_length */
static int tl(const uint8_t* b, size_t n, size_t* off, int* cls, int* tag, int* cmp, size_t* len) {
  if (*off >= n) return 0;
  uint8_t c = b[(*off)++];
  *cls = c >> 6;
  *cmp = (c & 0x20) != 0;
  *tag = c & 0x1f;
  if (*tag == 0x1f) {
    long v = 0;
    int shifted = 0, done = 0;
    while (*off < n) {
      if (shifted == 5) return 0;
      uint8_t x = b[(*off)++];
      v = (v << 7) | (x & 0x7f);
      shifted++;
      if (!(x & 0x80)) { done = 1; break; }
    }
    if (!done || v > 0x7fffffffL) return 0;
    if (v < 0x1f) return 0;
    *tag = (int)v;
  }
  if (*off >= n) return 0;
  c = b[(*off)++];
  if (!(c & 0x80)) { *len = c & 0x7f; return 1; }
  int nb = c & 0x7f;
  if (nb == 0) return 0;
  uint64_t l = 0;
  for (int i = 0; i < nb; i++) {
    if (*off >= n) return 0;
    c = b[(*off)++];
    if (l >= (1u << 23)) return 0;
    l = (l << 8) | c;
    if (l == 0) return 0;
  }
  if (l < 0x80) return 0;
  *len = (size_t)l;
  return 1;
}
static int der_int(const uint8_t* in, size_t n, size_t* off, uint8_t out32[32]) {
  int cls, tag, cmp;
  size_t len;
  memset(out32, 0, 32);
  if (*off == n) return 0;
  if (!tl(in, n, off, &cls, &tag, &cmp, &len)) return 0;
  if (cls != 0 || tag != 2 || cmp) return 0;
  if (len > n - *off) return 0;
  const uint8_t* v = in + *off;
  *off += len;
  if (len == 0) return 0;
  if (len > 1 && ((v[0] == 0 && !(v[1] & 0x80)) || (v[0] == 0xff && (v[1] & 0x80)))) return 0;
  if (v[0] & 0x80) return 1; /* negative -> 0 */
  size_t i = 0;
  while (i < len && v[i] == 0) i++;
  if (len - i > 32) return 1; /* >= 2^256 -> 0 (rejected like >= N) */
  memcpy(out32 + 32 - (len - i), v + i, len - i);
  return 1;
}
/* returns 1 ok (rest = *rest_len), 0 = asn1 error */
int oracle_der_parse(const uint8_t* sig, size_t n, uint8_t r32[32], uint8_t s32[32],
                     size_t* rest_len) {
  size_t off = 0, len;
  int cls, tag, cmp;
  if (n == 0) return 0;
  if (!tl(sig, n, &off, &cls, &tag, &cmp, &len)) return 0;
  if (cls != 0 || tag != 16 || !cmp) return 0;
  if (len > n - off) return 0;
  size_t ioff = 0;
  if (!der_int(sig + off, len, &ioff, r32)) return 0;
  if (!der_int(sig + off, len, &ioff, s32)) return 0;
  if (rest_len) *rest_len = n - off - len;
  return 1;
}

/* ------------------------------------------ authenticator-level (ECDSA) */
/* Status of Authenticator.VerifyMessageAuthenTag for an ECDSA role with a
 * known, valid key (crypto.go:79-89,113-126): 0 accept, 1 reject, 2 DER. */
int oracle_verify_ecdsa_role(const uint8_t qxy[64], const uint8_t* msg, size_t mlen,
                             const uint8_t* tag, size_t tlen) {
  static const uint8_t E[32] = {0xe3, 0xb0, 0xc4, 0x42, 0x98, 0xfc, 0x1c, 0x14, 0x9a, 0xfb, 0xf4,
                                0xc8, 0x99, 0x6f, 0xb9, 0x24, 0x27, 0xae, 0x41, 0xe4, 0x64, 0x9b,
                                0x93, 0x4c, 0xa4, 0x95, 0x99, 0x1b, 0x78, 0x52, 0xb8, 0x55};
  uint8_t r[32], s[32], e[32];
  size_t rest;
  if (!oracle_der_parse(tag, tlen, r, s, &rest)) return 2;
  for (size_t k = 0; k < 32; k++) e[k] = k < mlen ? msg[k] : E[k - mlen];
  int v = oracle_ecdsa_verify(qxy, e, r, s);
  return v == 1 ? 0 : 1;
}

/* USIG signature check with a matching epoch (usig-enclave.go:198-229):
 * 0 accept, 1 reject, 2 DER error, 3 trailing bytes. */
int oracle_verify_usig_sig(const uint8_t qxy[64], const uint8_t* msg, size_t mlen, uint64_t epoch,
                           uint64_t counter, const uint8_t* sig, size_t slen) {
  uint8_t buf[48], e[32], r[32], s[32];
  size_t rest;
  if (!oracle_der_parse(sig, slen, r, s, &rest)) return 2;
  if (rest) return 3;
  oracle_sha256(msg, mlen, buf);
  for (int k = 0; k < 8; k++) {
    buf[32 + k] = (uint8_t)(epoch >> (8 * k));
    buf[40 + k] = (uint8_t)(counter >> (8 * k));
  }
  oracle_sha256(buf, 48, e);
  return oracle_ecdsa_verify(qxy, e, r, s) == 1 ? 0 : 1;
}

/* ------------------------------------------------------ batch (threads) */
typedef struct {
  const uint8_t* qxy; /* nkeys x 64 */
  const uint8_t* e;
  const uint8_t* r;
  const uint8_t* s;
  const uint32_t* slot;
  uint8_t* out;
  size_t lo, hi;
} job_t;

static void* run_job(void* p) {
  job_t* j = (job_t*)p;
  for (size_t i = j->lo; i < j->hi; i++) {
    int v = oracle_ecdsa_verify(j->qxy + 64 * (size_t)j->slot[i], j->e + 32 * i, j->r + 32 * i,
                                j->s + 32 * i);
    j->out[i] = v == 1 ? 0 : (v < 0 ? 5 : 1);
  }
  return NULL;
}

/* out[i]: 0 accept, 1 reject, 5 invalid key */
int oracle_verify_prehashed_batch(const uint8_t* qxy, const uint8_t* e, const uint8_t* r,
                                  const uint8_t* s, const uint32_t* slot, size_t n, uint8_t* out,
                                  int nthreads) {
  pthread_once(&g_once, init_once);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){qxy, e, r, s, slot, out, n * t / nthreads, n * (t + 1) / nthreads};
    if (pthread_create(&th[t], NULL, run_job, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* Authenticator-level batch over REQUEST-style ECDSA items: msgs/tags are
 * packed with offsets (CSR).  out: status as oracle_verify_ecdsa_role. */
typedef struct {
  const uint8_t* qxy;
  const uint32_t* slot;
  const uint8_t* msgs;
  const uint64_t* moff;
  const uint8_t* tags;
  const uint64_t* toff;
  uint8_t* out;
  size_t lo, hi;
} ajob_t;

static void* run_ajob(void* p) {
  ajob_t* j = (ajob_t*)p;
  for (size_t i = j->lo; i < j->hi; i++)
    j->out[i] = (uint8_t)oracle_verify_ecdsa_role(
        j->qxy + 64 * (size_t)j->slot[i], j->msgs + j->moff[i], j->moff[i + 1] - j->moff[i],
        j->tags + j->toff[i], j->toff[i + 1] - j->toff[i]);
  return NULL;
}

int oracle_verify_ecdsa_role_batch(const uint8_t* qxy, const uint32_t* slot, const uint8_t* msgs,
                                   const uint64_t* moff, const uint8_t* tags,
                                   const uint64_t* toff, size_t n, uint8_t* out, int nthreads) {
  pthread_once(&g_once, init_once);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  ajob_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (ajob_t){qxy, slot, msgs, moff, tags, toff, out, n * t / nthreads,
                       n * (t + 1) / nthreads};
    if (pthread_create(&th[t], NULL, run_ajob, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}
