/*
 * oracle_check.c -- TEST INFRASTRUCTURE ONLY: a standalone driver of the CPU oracle, built with
 * AddressSanitizer + UndefinedBehaviorSanitizer (`make -C oracle asan`, SURVEY.md section 5
 * "Race detection / sanitizers").  It runs the synthetic workload of or_batch_run (counter-RNG
 * spawns and actions, auto-reset at done / the time limit) on one env id and prints the lane
 * capacity high-water marks; any out-of-bounds access, leak or undefined behaviour aborts the
 * run with a non-zero status.  tests/test_oracle.py runs it for every env id.
 *
 *   oracle_check_asan ENV LANES STEPS MAX_STEPS lo0 hi0 lo1 hi1 ...   (one lo/hi pair per draw)
 */
#include <stdio.h>
#include <stdlib.h>

#include "mrp_oracle.h"

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s ENV LANES STEPS MAX_STEPS lo0 hi0 ...\n", argv[0]);
        return 2;
    }
    const int env = atoi(argv[1]), lanes = atoi(argv[2]), steps = atoi(argv[3]), max_steps = atoi(argv[4]);
    const int nd = or_n_draws(env);
    if (nd <= 0 || argc != 5 + 2 * nd) {
        fprintf(stderr, "env %d takes %d draw bounds (lo hi pairs)\n", env, nd);
        return 2;
    }
    double* lo = (double*)malloc(sizeof(double) * (size_t)nd);
    double* hi = (double*)malloc(sizeof(double) * (size_t)nd);
    for (int d = 0; d < nd; ++d) { lo[d] = atof(argv[5 + 2 * d]); hi[d] = atof(argv[6 + 2 * d]); }
    int caps[8];
    const long n = or_batch_capacity(env, lanes, steps, 97, lo, hi, max_steps, 1, caps);
    free(lo);
    free(hi);
    if (n != (long)lanes * steps) {
        fprintf(stderr, "ran %ld env steps, expected %ld\n", n, (long)lanes * steps);
        return 1;
    }
    printf("{\"env\": %d, \"env_steps\": %ld, \"contacts\": %d, \"tree_node_id\": %d, \"move_buffer\": %d, "
           "\"island_bodies\": %d, \"island_contacts\": %d, \"toi_island_bodies\": %d, \"toi_island_contacts\": %d}\n",
           env, n, caps[0], caps[1], caps[2], caps[3], caps[4], caps[5], caps[6]);
    return 0;
}
