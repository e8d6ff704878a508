/* TEST INFRASTRUCTURE ONLY: drives the oracle under -fsanitize=address,undefined
 * ("race detection / sanitizers": the CPU restatement is
 * checked for out-of-bounds and undefined behaviour; the fixed-size stack
 * buffers of env_step_one are the main target).
 *
 *   oracle_san <dir>
 * reads   <dir>/cfg.bin    hftlob_env_cfg (raw struct, packed by hftlob.layout)
 *         <dir>/msgs.bin   int32 [n_data_rows][8]
 *         <dir>/init.bin   int32 [n_windows][init_rec_words]
 *         <dir>/keys.bin   uint32 [n_env][2] reset keys
 *         <dir>/book.bin   int32 [book_env][book_msg][8] engine messages
 *         <dir>/params.txt n_env n_steps master0 master1 book_env book_msg
 * writes  <dir>/state.bin  int32 [n_env][rec_words] after reset, one env_step (with info) and
 *                          an n_steps rollout
 *         <dir>/info.bin   int32 [n_env][info_words] of that env_step
 *         <dir>/book_out.bin asks, bids, trades, best_asks, best_bids of oracle_book_process
 * tests/test_oracle_sanitize.py compares them with the -O2 oracle's results. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hftlob.h"

int oracle_env_reset(const hftlob_env_cfg* c, int n_env, const uint32_t* keys, const int32_t* init_states,
                     int32_t* state, float* obs);
int oracle_env_step(const hftlob_env_cfg* c, int n_env, const uint32_t* keys, const int32_t* actions,
                    const int32_t* msg_data, const int32_t* init_states, int32_t* state, float* obs, float* rew,
                    int32_t* done_all, int32_t* dones, int32_t* info);
void oracle_sample_actions(const hftlob_env_cfg* c, int n_env, const uint32_t* keys, int32_t* actions);
int oracle_rollout_sampled(const hftlob_env_cfg* c, int n_env, int key_e0, int key_n, int n_steps, uint32_t* master,
                           const int32_t* msg_data, const int32_t* init_states, int32_t* state);
int oracle_book_process(const hftlob_lob_cfg* c, int n_env, int n_msg, const uint32_t* keys, const int32_t* msgs,
                        int32_t* asks, int32_t* bids, int32_t* trades, int32_t* best_asks, int32_t* best_bids);

static void* slurp(const char* dir, const char* name, size_t want) {
    char p[4096];
    snprintf(p, sizeof p, "%s/%s", dir, name);
    FILE* f = fopen(p, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", p); exit(2); }
    void* buf = malloc(want ? want : 1);
    if (fread(buf, 1, want, f) != want) { fprintf(stderr, "short read %s\n", p); exit(2); }
    fclose(f);
    return buf;
}

static void dump(const char* dir, const char* name, const void* buf, size_t n) {
    char p[4096];
    snprintf(p, sizeof p, "%s/%s", dir, name);
    FILE* f = fopen(p, "wb");
    if (!f || fwrite(buf, 1, n, f) != n) { fprintf(stderr, "cannot write %s\n", p); exit(2); }
    fclose(f);
}

int main(int argc, char** argv) {
    if (argc != 2) { fprintf(stderr, "usage: %s <dir>\n", argv[0]); return 2; }
    const char* dir = argv[1];
    hftlob_env_cfg* c = (hftlob_env_cfg*)slurp(dir, "cfg.bin", sizeof(hftlob_env_cfg));
    int n_env, n_steps, book_env, book_msg;
    unsigned m0, m1;
    char p[4096];
    snprintf(p, sizeof p, "%s/params.txt", dir);
    FILE* f = fopen(p, "r");
    if (!f || fscanf(f, "%d %d %u %u %d %d", &n_env, &n_steps, &m0, &m1, &book_env, &book_msg) != 6) return 2;
    fclose(f);
    int32_t* msgs = (int32_t*)slurp(dir, "msgs.bin", sizeof(int32_t) * 8 * (size_t)c->n_data_rows);
    int32_t* init = (int32_t*)slurp(dir, "init.bin", sizeof(int32_t) * (size_t)c->n_windows * c->init_rec_words);
    uint32_t* keys = (uint32_t*)slurp(dir, "keys.bin", sizeof(uint32_t) * 2 * (size_t)n_env);
    int32_t* state = (int32_t*)calloc((size_t)n_env * c->rec_words, sizeof(int32_t));
    float* obs = (float*)calloc((size_t)n_env * c->n_agents * c->obs_stride, sizeof(float));
    float* rew = (float*)calloc((size_t)n_env * c->n_agents, sizeof(float));
    int32_t* da = (int32_t*)calloc((size_t)n_env, sizeof(int32_t));
    int32_t* dn = (int32_t*)calloc((size_t)n_env * c->n_agents, sizeof(int32_t));
    int32_t* info = (int32_t*)calloc((size_t)n_env * c->info_words, sizeof(int32_t));
    int32_t* acts = (int32_t*)calloc((size_t)n_env * c->action_words, sizeof(int32_t));
    if (oracle_env_reset(c, n_env, keys, init, state, obs)) return 3;
    oracle_sample_actions(c, n_env, keys, acts);
    if (oracle_env_step(c, n_env, keys, acts, msgs, init, state, obs, rew, da, dn, info)) return 3;
    uint32_t master[2] = {m0, m1};
    if (oracle_rollout_sampled(c, n_env, 0, n_env, n_steps, master, msgs, init, state)) return 3;
    dump(dir, "state.bin", state, sizeof(int32_t) * (size_t)n_env * c->rec_words);
    dump(dir, "info.bin", info, sizeof(int32_t) * (size_t)n_env * c->info_words);
    /* engine operator over a batch of message streams */
    const int nO = c->lob.n_orders, nT = c->lob.n_trades;
    int32_t* bm = (int32_t*)slurp(dir, "book.bin", sizeof(int32_t) * 8 * (size_t)book_env * book_msg);
    size_t na = (size_t)book_env * nO * 6, nt = (size_t)book_env * nT * 8, nb = (size_t)book_env * book_msg * 2;
    int32_t* out = (int32_t*)malloc(sizeof(int32_t) * (2 * na + nt + 2 * nb));
    for (size_t i = 0; i < 2 * na + nt; ++i) out[i] = -1;
    uint32_t* bk = (uint32_t*)calloc((size_t)book_env * 2, sizeof(uint32_t));
    if (oracle_book_process(&c->lob, book_env, book_msg, bk, bm, out, out + na, out + 2 * na, out + 2 * na + nt,
                            out + 2 * na + nt + nb))
        return 3;
    dump(dir, "book_out.bin", out, sizeof(int32_t) * (2 * na + nt + 2 * nb));
    free(c); free(msgs); free(init); free(keys); free(state); free(obs); free(rew); free(da); free(dn);
    free(info); free(acts); free(bm); free(out); free(bk);
    return 0;
}
