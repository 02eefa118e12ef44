/*
 * mgpu_shard.c -- a C host of libtlsrec.so across GPUs: one process per GPU,
 * the key table broadcast from rank 0 over RCCL (xGMI), a contiguous record
 * shard per rank, no data-path collective (SURVEY.md
 * 8(e)).  The sequence a multi-GPU C terminator would run:
 *
 *   rank 0: key material (tlsrec_key_material[], 64 B per slot) -> device
 *   all:    ncclBroadcast(keys, root 0)                  -- the only exchange
 *   all:    tlsrec_keytab_load(kt, 0, n, d_keys, keys_on_device = 1)
 *   all:    tlsrec_shard_bounds(records, rank, world) -> [start, start+count)
 *   all:    tlsrec_batch_encrypt / _decrypt on the shard (records never
 *           leave their GPU)
 *   all:    ncclAllReduce of [records, ok] status counts (control plane)
 *
 *   mgpu_shard [world] [records] [content]
 *
 * Forks `world` processes (rank r on device r % device count; world 1 runs
 * in this process); the parent touches no GPU.  Each rank checks that its key table equals rank 0's and
 * that every record of its shard round-trips (encrypt, decrypt, plaintext
 * and statuses compared).  Rank 0 prints one JSON line; exit status 0 = pass.
 */
#define _POSIX_C_SOURCE 200809L
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "tlsrec.h"

#define NKEYS 256u

static uint64_t splitmix(uint64_t *s)
{
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* rank 0's key table: AES-256-GCM and ChaCha20-Poly1305 alternating, TLS 1.3 */
static void make_keys(tlsrec_key_material *km)
{
    uint64_t s = 0x6b657973ull;
    memset(km, 0, NKEYS * sizeof(*km));
    for (uint32_t i = 0; i < NKEYS; i++) {
        km[i].cipher = (i & 1) ? TLSREC_CIPHER_CHACHA20_POLY1305 : TLSREC_CIPHER_AES_256_GCM;
        km[i].tls_minor = 4;
        km[i].fixed_ivlen = 12;
        km[i].taglen = 16;
        for (int b = 0; b < 32; b++) km[i].key[b] = (uint8_t) splitmix(&s);
        for (int b = 0; b < 12; b++) km[i].iv[b] = (uint8_t) splitmix(&s);
    }
}

static uint8_t content_byte(uint64_t rec, uint32_t j)
{
    uint64_t s = rec * 0x100000001b3ull + j / 8;
    return (uint8_t) (splitmix(&s) >> (8 * (j % 8)));
}

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "rank %d: %s failed\n", rank, #x); return 2; } } while (0)
#define CN(x) do { if ((x) != ncclSuccess) { fprintf(stderr, "rank %d: %s failed\n", rank, #x); return 2; } } while (0)
#define CT(x) do { int rc_ = (x); if (rc_ != 0) { fprintf(stderr, "rank %d: %s = %d\n", rank, #x, rc_); return 2; } } while (0)

static int run_rank(int rank, int world, ncclUniqueId id, uint64_t n, uint32_t content)
{
    int ndev = 0;
    CK(hipGetDeviceCount(&ndev));
    if (ndev < 1) return 2;
    CK(hipSetDevice(rank % ndev));
    ncclComm_t comm;
    CN(ncclCommInitRank(&comm, world, id, rank));
    hipStream_t st;
    CK(hipStreamCreate(&st));

    /* ---- key table: rank 0's material, broadcast, loaded from the device ---- */
    tlsrec_key_material *km = calloc(NKEYS, sizeof(*km)), *ref = calloc(NKEYS, sizeof(*ref));
    make_keys(ref);
    if (rank == 0) memcpy(km, ref, NKEYS * sizeof(*km));
    void *d_keys = NULL;
    CK(hipMalloc(&d_keys, NKEYS * sizeof(*km)));
    CK(hipMemcpy(d_keys, km, NKEYS * sizeof(*km), hipMemcpyHostToDevice));
    CN(ncclBroadcast(d_keys, d_keys, NKEYS * sizeof(*km), ncclUint8, 0, comm, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(km, d_keys, NKEYS * sizeof(*km), hipMemcpyDeviceToHost));
    const int keys_match = memcmp(km, ref, NKEYS * sizeof(*km)) == 0;
    tlsrec_keytab *kt = NULL;
    CT(tlsrec_keytab_create(&kt, NKEYS));
    CT(tlsrec_keytab_load(kt, 0, NKEYS, (const tlsrec_key_material *) d_keys, 1, st));

    /* ---- this rank's shard of the global record stream ---- */
    uint64_t start = 0, count = 0;
    CT(tlsrec_shard_bounds(n, (uint32_t) rank, (uint32_t) world, &start, &count));
    const uint32_t stride = (content + 1 + 16 + 127) / 128 * 128;    /* TLS 1.3: type byte + tag */
    uint8_t *h_arena = calloc(count ? count : 1, stride);
    tlsrec_batch_rec *h_recs = calloc(count ? count : 1, sizeof(*h_recs));
    tlsrec_batch_res *h_res = calloc(count ? count : 1, sizeof(*h_res));
    for (uint64_t i = 0; i < count; i++) {
        const uint64_t g = start + i;                     /* global record index = sequence number */
        tlsrec_batch_rec *r = &h_recs[i];
        r->buf_off = i * stride;
        r->buf_len = stride;
        r->data_offset = 0;
        r->data_len = content;
        r->slot = (uint32_t) (g % NKEYS);
        for (int b = 0; b < 8; b++) r->ctr[b] = (uint8_t) ((g / NKEYS) >> (56 - 8 * b));
        r->type = 23;
        r->ver[0] = r->ver[1] = 3;
        for (uint32_t j = 0; j < content; j++) h_arena[i * stride + j] = content_byte(g, j);
    }
    uint8_t *d_arena = NULL;
    tlsrec_batch_rec *d_recs = NULL;
    tlsrec_batch_res *d_res = NULL;
    CK(hipMalloc((void **) &d_arena, (count ? count : 1) * stride));
    CK(hipMalloc((void **) &d_recs, (count ? count : 1) * sizeof(*d_recs)));
    CK(hipMalloc((void **) &d_res, (count ? count : 1) * sizeof(*d_res)));
    CK(hipMemcpy(d_arena, h_arena, count * stride, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_recs, h_recs, count * sizeof(*d_recs), hipMemcpyHostToDevice));
    CT(tlsrec_batch_encrypt(kt, d_recs, d_res, (uint32_t) count, d_arena, d_arena, 0, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h_res, d_res, count * sizeof(*h_res), hipMemcpyDeviceToHost));
    uint64_t enc_ok = 0;
    for (uint64_t i = 0; i < count; i++) {
        enc_ok += h_res[i].status == 0;
        h_recs[i].data_offset = h_res[i].data_offset;      /* the protected record, as encrypt left it */
        h_recs[i].data_len = h_res[i].data_len;
        h_recs[i].type = h_res[i].type;
    }
    CK(hipMemcpy(d_recs, h_recs, count * sizeof(*d_recs), hipMemcpyHostToDevice));
    CK(hipMemset(d_res, 0x55, count * sizeof(*d_res)));   /* every result must be written */
    CT(tlsrec_batch_decrypt(kt, d_recs, d_res, (uint32_t) count, d_arena, d_arena, 0, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h_res, d_res, count * sizeof(*h_res), hipMemcpyDeviceToHost));
    uint8_t *back = malloc((count ? count : 1) * stride);
    CK(hipMemcpy(back, d_arena, count * stride, hipMemcpyDeviceToHost));
    uint64_t ok = 0;
    for (uint64_t i = 0; i < count; i++) {
        int good = h_res[i].status == 0 && h_res[i].data_len == content && h_res[i].type == 23;
        for (uint32_t j = 0; good && j < content; j++)
            good = back[i * stride + h_res[i].data_offset + j] == content_byte(start + i, j);
        ok += (uint64_t) good;
    }

    /* ---- control plane: status counts summed over ranks ---- */
    uint64_t tot[4] = { count, ok, enc_ok, (uint64_t) keys_match }, *d_tot = NULL;
    CK(hipMalloc((void **) &d_tot, sizeof(tot)));
    CK(hipMemcpy(d_tot, tot, sizeof(tot), hipMemcpyHostToDevice));
    CN(ncclAllReduce(d_tot, d_tot, 4, ncclUint64, ncclSum, comm, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(tot, d_tot, sizeof(tot), hipMemcpyDeviceToHost));
    const int pass = tot[0] == n && tot[1] == n && tot[2] == n && tot[3] == (uint64_t) world;
    if (!pass)
        fprintf(stderr, "rank %d: shard [%llu, +%llu) encrypt ok %llu, round trip ok %llu, keys %s; first status %d len %u\n",
                rank, (unsigned long long) start, (unsigned long long) count, (unsigned long long) enc_ok,
                (unsigned long long) ok, keys_match ? "match" : "DIFFER", count ? h_res[0].status : 0,
                count ? h_res[0].data_len : 0);
    if (rank == 0)
        printf("{\"world\": %d, \"records\": %llu, \"round_trip_ok\": %llu, \"encrypt_ok\": %llu, "
               "\"ranks_with_rank0_keys\": %llu, \"shard0\": [%llu, %llu], \"pass\": %s}\n",
               world, (unsigned long long) tot[0], (unsigned long long) tot[1], (unsigned long long) tot[2],
               (unsigned long long) tot[3], (unsigned long long) start, (unsigned long long) count,
               pass ? "true" : "false");
    tlsrec_keytab_free(kt);
    (void) hipFree(d_arena);
    (void) hipFree(d_recs);
    (void) hipFree(d_res);
    (void) hipFree(d_tot);
    (void) hipFree(d_keys);
    ncclCommDestroy(comm);
    free(km); free(ref); free(h_arena); free(h_recs); free(h_res); free(back);
    return pass ? 0 : 1;
}

int main(int argc, char **argv)
{
    const int world = argc > 1 ? atoi(argv[1]) : 1;
    const uint64_t n = argc > 2 ? strtoull(argv[2], NULL, 10) : 4096;
    const uint32_t content = argc > 3 ? (uint32_t) atoi(argv[3]) : 1400;
    if (world < 1 || world > 16 || content > 16383) return 2;
    if (world == 1) {   /* one rank: in this process */
        ncclUniqueId id;
        if (ncclGetUniqueId(&id) != ncclSuccess) return 2;
        return run_rank(0, 1, id, n, content);
    }
    /* rank 0 makes the RCCL id and hands it to the others through a pipe:
     * the parent process never initialises the GPU */
    int fds[2];
    if (pipe(fds) != 0) return 2;
    pid_t pids[16];
    for (int r = 0; r < world; r++) {
        pids[r] = fork();
        if (pids[r] < 0) return 2;
        if (pids[r] == 0) {
            ncclUniqueId id;
            if (r == 0) {
                if (ncclGetUniqueId(&id) != ncclSuccess) _exit(2);
                for (int k = 1; k < world; k++)
                    if (write(fds[1], &id, sizeof(id)) != (ssize_t) sizeof(id)) _exit(2);
            } else if (read(fds[0], &id, sizeof(id)) != (ssize_t) sizeof(id)) {
                _exit(2);
            }
            const int rc = run_rank(r, world, id, n, content);
            fflush(stdout);
            fflush(stderr);
            _exit(rc);
        }
    }
    int fail = 0;
    for (int r = 0; r < world; r++) {
        int stt = 0;
        if (waitpid(pids[r], &stt, 0) < 0 || !WIFEXITED(stt) || WEXITSTATUS(stt) != 0) fail = 1;
    }
    return fail;
}
