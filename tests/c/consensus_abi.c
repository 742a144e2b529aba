/* A plain C caller of the single-matrix C-ABI (include/pcx.h) -- what a non-Python binding
 * (a Simulator.jl ccall, a C++ service) does: no Python, no torch, host buffers.
 *
 *   consensus_abi IN OUT WORLD [DEVICES]
 *
 * IN: int64 N, E, has_rep, has_bounds; f64 reports[N][E]; f64 rep[N] (if has_rep);
 *     u8 scaled[E], f64 lo[E], f64 hi[E] (if has_bounds).
 * WORLD == 1: pcx_create(0) + pcx_consensus_f64.  WORLD > 1: an in-process group of WORLD
 * virtual ranks (threads, contexts from pcx_create_grouped), each passing only its rows.
 * DEVICES ("0,0,1", WORLD ids): ONE call on a pcx_create_devices context with the whole
 * matrix -- the library shards the rows over the listed devices itself.
 * OUT: f64 agents[8][N] (rows concatenated over ranks), events[9][E] (rank 0; every rank's
 * must be bit-identical), filled[N][E], then participation, avg_certainty, branch, flags,
 * n_hard, sel_passes as f64.  Exit status 0 = success. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcx.h"

static int64_t N, E, has_rep, has_bounds;
static double *reports, *rep, *lo, *hi;
static uint8_t* scaled;
static double *agents, *events_all, *filled;
static pcx_result results[64];
static pcx_group* group;
static int world;

static void* rank_main(void* arg) {
    const int r = (int)(intptr_t)arg;
    const int64_t base = N / world, rem = N % world;
    const int64_t cnt = base + (r < rem), off = r * base + (r < rem ? r : rem);
    pcx_ctx* ctx = world == 1 ? pcx_create(0) : pcx_create_grouped(0, group, r);
    if (!ctx) {
        fprintf(stderr, "rank %d: context: %s\n", r, pcx_last_error());
        return (void*)1;
    }
    pcx_problem p;
    memset(&p, 0, sizeof p);
    p.n_rows = cnt;
    p.n_events = E;
    p.n_total = N;
    p.row_offset = off;
    p.reports = reports + off * E;
    p.reputation = has_rep ? rep : NULL;
    p.scaled = has_bounds ? scaled : NULL;
    p.lo = has_bounds ? lo : NULL;
    p.hi = has_bounds ? hi : NULL;
    p.catch_tolerance = 0.1;
    p.alpha = 0.1;
    p.algorithm = PCX_ALG_PCA;
    p.max_components = 5;
    p.variance_threshold = 0.9;
    p.mem_kind = PCX_MEM_HOST;
    pcx_result* res = &results[r];
    memset(res, 0, sizeof *res);
    double** av[8] = {&res->old_rep, &res->this_rep, &res->smooth_rep, &res->scores, &res->na_row,
                      &res->participation_rows, &res->relative_part, &res->reporter_bonus};
    for (int k = 0; k < 8; k++) *av[k] = agents + k * N + off;
    double** ev[9] = {&res->adj_first_loadings, &res->outcomes_raw, &res->outcomes_adjusted, &res->outcomes_final,
                      &res->certainty, &res->consensus_reward, &res->nas_filled, &res->participation_columns,
                      &res->author_bonus};
    for (int k = 0; k < 9; k++) *ev[k] = events_all + ((int64_t)r * 9 + k) * E;
    res->filled = filled + off * E;
    const int rc = pcx_consensus_f64(ctx, &p, res);
    if (rc) fprintf(stderr, "rank %d: pcx_consensus_f64 = %d: %s\n", r, rc, pcx_last_error());
    pcx_destroy(ctx);
    return (void*)(intptr_t)(rc != 0);
}

/* the whole matrix in one call on a multi-device context (pcx_create_devices) */
static int run_devices(const char* list) {
    int ids[64], n = 0;
    for (const char* c = list; *c && n < 64;) {
        ids[n++] = atoi(c);
        while (*c && *c != ',') c++;
        if (*c == ',') c++;
    }
    if (n != world) return 2;
    pcx_ctx* ctx = pcx_create_devices(n, ids);
    if (!ctx) {
        fprintf(stderr, "pcx_create_devices: %s\n", pcx_last_error());
        return 1;
    }
    pcx_problem p;
    memset(&p, 0, sizeof p);
    p.n_rows = N;
    p.n_events = E;
    p.n_total = N;
    p.reports = reports;
    p.reputation = has_rep ? rep : NULL;
    p.scaled = has_bounds ? scaled : NULL;
    p.lo = has_bounds ? lo : NULL;
    p.hi = has_bounds ? hi : NULL;
    p.catch_tolerance = 0.1;
    p.alpha = 0.1;
    p.algorithm = PCX_ALG_PCA;
    p.max_components = 5;
    p.variance_threshold = 0.9;
    p.mem_kind = PCX_MEM_HOST;
    pcx_result* res = &results[0];
    memset(res, 0, sizeof *res);
    double** av[8] = {&res->old_rep, &res->this_rep, &res->smooth_rep, &res->scores, &res->na_row,
                      &res->participation_rows, &res->relative_part, &res->reporter_bonus};
    for (int k = 0; k < 8; k++) *av[k] = agents + k * N;
    double** ev[9] = {&res->adj_first_loadings, &res->outcomes_raw, &res->outcomes_adjusted, &res->outcomes_final,
                      &res->certainty, &res->consensus_reward, &res->nas_filled, &res->participation_columns,
                      &res->author_bonus};
    for (int k = 0; k < 9; k++) *ev[k] = events_all + k * E;
    res->filled = filled;
    const int rc = pcx_consensus_f64(ctx, &p, res);
    if (rc) fprintf(stderr, "pcx_consensus_f64 (devices %s) = %d: %s\n", list, rc, pcx_last_error());
    if (!rc && pcx_ctx_world(ctx) != n) {
        fprintf(stderr, "pcx_ctx_world = %d, expected %d\n", pcx_ctx_world(ctx), n);
        pcx_destroy(ctx);
        return 1;
    }
    pcx_destroy(ctx);
    return rc != 0;
}

/* WORLD threads, one grouped context each, every rank passing only its rows */
static int run_ranks(void) {
    if (world > 1) group = pcx_group_create(world);
    pthread_t th[64];
    for (int r = 0; r < world; r++) pthread_create(&th[r], NULL, rank_main, (void*)(intptr_t)r);
    int fail = 0;
    for (int r = 0; r < world; r++) {
        void* v;
        pthread_join(th[r], &v);
        fail |= v != NULL;
    }
    if (group) pcx_group_destroy(group);
    if (fail) return 1;
    for (int r = 1; r < world; r++) /* event outputs identical on every rank */
        if (memcmp(events_all, events_all + (int64_t)r * 9 * E, 9 * E * 8)) {
            fprintf(stderr, "rank %d event outputs differ from rank 0\n", r);
            return 4;
        }
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 4 && argc != 5) return 2;
    world = atoi(argv[3]);
    if (world < 1 || world > 64) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int64_t hdr[4];
    if (fread(hdr, 8, 4, f) != 4) return 2;
    N = hdr[0], E = hdr[1], has_rep = hdr[2], has_bounds = hdr[3];
    reports = malloc(N * E * 8);
    rep = malloc(N * 8);
    scaled = malloc(E);
    lo = malloc(E * 8);
    hi = malloc(E * 8);
    agents = malloc(8 * N * 8);
    events_all = malloc((size_t)world * 9 * E * 8);
    filled = malloc(N * E * 8);
    size_t ok = fread(reports, 8, N * E, f) == (size_t)(N * E);
    if (has_rep) ok &= fread(rep, 8, N, f) == (size_t)N;
    if (has_bounds) ok &= fread(scaled, 1, E, f) == (size_t)E && fread(lo, 8, E, f) == (size_t)E &&
                          fread(hi, 8, E, f) == (size_t)E;
    fclose(f);
    if (!ok) return 2;
    if (pcx_abi_version() != PCX_ABI_VERSION) return 3;
    const int rc = argc == 5 ? run_devices(argv[4]) : run_ranks();
    if (rc) return rc;
    FILE* o = fopen(argv[2], "wb");
    fwrite(agents, 8, 8 * N, o);
    fwrite(events_all, 8, 9 * E, o);
    fwrite(filled, 8, N * E, o);
    const double sc[6] = {results[0].participation, results[0].avg_certainty, results[0].branch, results[0].flags,
                          results[0].n_hard, results[0].sel_passes};
    fwrite(sc, 8, 6, o);
    fclose(o);
    printf("ok world=%d%s branch=%d n_hard=%d sel_passes=%d\n", world, argc == 5 ? " (one call, pcx_create_devices)" : "",
           results[0].branch, results[0].n_hard,
           results[0].sel_passes);
    return 0;
}
