/*
 * ct_walk.c — a plain C caller of the C-ABI (include/cilium_hip.h), the way the Go
 * agent's cgo glue calls it.  It fills a CT4 map with N distinct entries, attaches
 * the map to an endpoint (so it becomes the device-resident table), then walks it
 * with cv_map_get_next_key from NULL to -ENOENT -- the ctmap dump walk
 * (pkg/maps/ctmap/ctmap.go:196-230 over pkg/bpf/bpf.go:218-245) -- and times the
 * walk.  Prints one line: entries visited unique walk_s.
 *
 * Built by cilium_amd/build.py into tests/_bin/ct_walk; run by tests/test_gpu_parity.py.
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/cilium_hip.h"

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 0) : 1u << 20;
    cv_ctx *c;
    if (cv_open(0, &c)) { fprintf(stderr, "cv_open failed\n"); return 2; }
    int ct, pol;
    if (cv_map_create(c, CV_MAP_LRU_HASH, 14, 56, n + 1024, 0, &ct) ||
        cv_map_create(c, CV_MAP_HASH, 8, 24, 1024, 0, &pol)) { fprintf(stderr, "map create\n"); return 2; }
    uint8_t *keys = calloc(n, 14), *vals = calloc(n, 56);
    for (uint32_t i = 0; i < n; ++i) {           /* ipv4_ct_tuple {daddr = i, saddr, ports, TCP, IN} */
        uint8_t *k = keys + (size_t)i * 14;
        memcpy(k, &i, 4);
        k[4] = 10; k[7] = 1;
        k[8] = 0; k[9] = 80;
        k[10] = (uint8_t)(i >> 8); k[11] = (uint8_t)i;
        k[12] = 6; k[13] = 1;
        uint32_t life = 1000 + (i & 1023);
        memcpy(vals + (size_t)i * 56 + 32, &life, 4);
    }
    uint32_t done = 0;
    if (cv_map_update_batch(c, ct, keys, vals, n, CV_ANY, &done) || done != n) { fprintf(stderr, "fill\n"); return 2; }
    if (cv_endpoint_add(c, 1, 0x1000, pol, ct) < 0) { fprintf(stderr, "endpoint\n"); return 2; }
    uint32_t cnt = 0;
    cv_map_count(c, ct, &cnt);
    uint8_t *seen = calloc(n, 1);
    uint8_t cur[14], nxt[14];
    uint32_t visited = 0, unique = 0;
    const double t0 = now_s();
    int rc = cv_map_get_next_key(c, ct, NULL, nxt);
    while (rc == 0) {
        uint32_t i;
        memcpy(&i, nxt, 4);
        ++visited;
        if (i < n && !seen[i]) { seen[i] = 1; ++unique; }
        memcpy(cur, nxt, 14);
        rc = cv_map_get_next_key(c, ct, cur, nxt);
    }
    const double t1 = now_s();
    printf("count %u entries %u visited %u unique %u end %d walk_s %.4f\n", cnt, n, visited, unique, rc, t1 - t0);
    cv_close(c);
    return rc == -ENOENT ? 0 : 1;
}
