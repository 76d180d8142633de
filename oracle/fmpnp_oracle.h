/* fmpnp_oracle.h -- CPU restatement of the reference LM loop (TEST INFRASTRUCTURE).
 * See fmpnp_oracle.c for scope and citations. */
#ifndef FMPNP_ORACLE_H
#define FMPNP_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_SQUARED = 0, ORC_HUBER = 1, ORC_CAUCHY = 2, ORC_GEMAN_MCCLURE = 3, ORC_BARRON = 4 };
enum { ORC_OK = 0, ORC_NO_SUPPORT = 1, ORC_NAN = 2, ORC_NO_SUPPORT_TRIAL = 4 };
enum { ORC_NEAREST = 0, ORC_BILINEAR = 1 }; /* sampling: the reference's NN, or the bilinear extension */

typedef struct {
    const double *fmap, *gx, *gy; /* [C][Hf][Wf] fp64 (already channel-sliced) */
    int C, Hf, Wf;
    const double *fref;           /* [N][ld_ref] fp64, first C columns used */
    int ld_ref;
    const double *pts;            /* [N][3] */
    int N;
    double K[9], R0[9], t0[3];
    int im_w, im_h;
} orc_problem;

typedef struct {
    int n_iters;
    double lambda0;
    int use_ratio;
    double ratio_threshold;
    int loss;
    double barron_alpha;
    int sampling;                 /* ORC_NEAREST (the reference) or ORC_BILINEAR (extension) */
} orc_options;

typedef struct {
    double R[9], t[3];
    double initial_cost, best_cost, final_lambda, final_lr;
    int best_num_inliers, status, n_evals, n_steps, n_accepted, has_best;
} orc_result;

typedef struct { /* optional per-eval / per-step trace, capacity cap entries each */
    int cap;
    double *R, *t, *cost;        /* per eval: [cap][9], [cap][3], [cap] */
    int *n_supported, *n_kept;   /* per eval */
    double *g, *H, *lam, *lr, *delta; /* per step: [cap][6], [cap][36], [cap], [cap], [cap][6] */
} orc_trace;

int orc_forward(const orc_problem *pb, const orc_options *op, orc_result *res, orc_trace *tr);
double orc_compute_cost(const orc_problem *pb, double ratio_threshold, const double R[9], const double t[3]);
int orc_find_inliers(const orc_problem *pb, const double R[9], const double t[3], int loss, double alpha,
                     double threshold, unsigned char *mask, double *cost_out);
void orc_sobel(const double *x, int C, int H, int W, double *gx, double *gy);
int orc_forward_batch(const orc_problem *pbs, int n, const orc_options *op, orc_result *res, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
