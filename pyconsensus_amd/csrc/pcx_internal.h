// pcx_internal.h -- declarations shared by the libpcx translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/pcx.h"

namespace pcx {

// Kernel arguments of the batched round kernel (by value).
struct BatchArgs {
    int64_t B;
    int N, E, ES;
    const double* reports;
    const double* reputation;
    const uint8_t* scaled;
    const double* lo;
    const double* hi;
    int bounds_shared;
    int int_dtype;
    int algorithm;
    int max_components;       // big-five
    double variance_threshold;  // fixed-variance
    const double* aux_scores;   // cokurtosis [B][N]
    double hierarchy_threshold;  // hierarchical
    double cluster_threshold;    // clusterfeck (<= 0: log10(E)/1.77 rule)
    int kmeans_k, kmeans_restarts;
    const int32_t* kmeans_init;  // k-means [B][restarts][k]
    double catch_tol;
    double alpha;
    double *old_rep, *this_rep, *smooth_rep, *scores, *na_row, *participation_rows, *relative_part,
        *reporter_bonus;
    double *adj_first_loadings, *outcomes_raw, *outcomes_adjusted, *outcomes_final, *certainty,
        *consensus_reward, *nas_filled, *participation_columns, *author_bonus;
    double *participation, *avg_certainty;
    int32_t *branch, *flags, *pi_iters, *components;
    double *original, *filled;
    long long* stamps;  // diagnostic phase clocks [B][16] (PCX_STAMPS), normally NULL
};

size_t batched_lds_bytes(int N, int E);
hipError_t launch_batched(const BatchArgs& a, hipStream_t stream);

// single-matrix path: launch one stage (pcx_matrix.hip)
hipError_t mat_stage(pcx_mat& m, int stage, hipStream_t stream, std::string& err);

}  // namespace pcx
