/* The walk gate ("Next round" item 1): how much independent work
 * hides inside one states-walk chain.
 *
 * Input: a chain file of int32 symbols (ctx << 16 | folded residual as u16),
 * one (GOP, slice, plane group) chain in coding order, frames back to back,
 * with the symbol count of each frame (tools/gate/walk_gate.py writes both
 * from the oracle's ffv1o_slice_symbols).
 *
 * (a) context windows: for windows of W symbols, the largest context's share
 *     and the makespan of list-scheduling the window's contexts on P workers
 *     (each worker walks whole contexts), as a multiple of W / P;
 * (b) trajectory merging: at every frame boundary, every (context, slot)
 *     state trajectory restarted from a wrong state (every other state, and
 *     the state one frame stale) against the true one: the decisions of the
 *     frame before the two merge.
 *
 * Decisions per symbol follow put_symbol_inline (ffv1enc.c:185-231):
 * slot 0 (zero), 1 + min(i, 9) (exponent), 22 + min(i, 9) (mantissa),
 * 11 + min(e, 10) (sign).  The transition tables are the custom ones the
 * encoder installs (ffv1enc.c:1309-1315), taken from the oracle source.
 *
 * Build: gcc -O2 -o tools/gate/walk_gate tools/gate/walk_gate.c -lm
 * (includes oracle/ffv1_oracle.c for its tables: a measurement tool, never
 * part of the product). */
#include "../../oracle/ffv1_oracle.c"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint8_t slot, bit;
} dec_t;

static int decisions(int v, dec_t *d)
{
    int n = 0;
    if (v == 0) {
        d[n++] = (dec_t){0, 1};
        return n;
    }
    unsigned a = v < 0 ? -v : v;
    int e = 31 - __builtin_clz(a);
    d[n++] = (dec_t){0, 0};
    for (int i = 0; i < e; i++)
        d[n++] = (dec_t){(uint8_t)(1 + (i < 9 ? i : 9)), 1};
    d[n++] = (dec_t){(uint8_t)(1 + (e < 9 ? e : 9)), 0};
    for (int i = e - 1; i >= 0; i--)
        d[n++] = (dec_t){(uint8_t)(22 + (i < 9 ? i : 9)), (uint8_t)((a >> i) & 1)};
    d[n++] = (dec_t){(uint8_t)(11 + (e < 10 ? e : 10)), (uint8_t)(v < 0)};
    return n;
}

static int cmp_desc(const void *a, const void *b)
{
    int x = *(const int *)a, y = *(const int *)b;
    return y - x;
}

/* list scheduling, largest first, on P workers: the makespan */
static int lpt(int *cnt, int n, int P)
{
    int load[64] = {0};
    qsort(cnt, n, sizeof(int), cmp_desc);
    for (int i = 0; i < n; i++) {
        int m = 0;
        for (int p = 1; p < P; p++)
            if (load[p] < load[m])
                m = p;
        load[m] += cnt[i];
    }
    int mx = 0;
    for (int p = 0; p < P; p++)
        if (load[p] > mx)
            mx = load[p];
    return mx;
}

#define NCTX 8192

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: walk_gate chain.bin frames.txt\n");
        return 2;
    }
    FILE *f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    long nb = ftell(f);
    fseek(f, 0, SEEK_SET);
    int64_t n = nb / 4;
    int32_t *sym = malloc(nb);
    if (fread(sym, 4, n, f) != (size_t)n)
        return 1;
    fclose(f);
    int64_t fr[64];
    int nfr = 0;
    FILE *g = fopen(argv[2], "r");
    while (nfr < 64 && fscanf(g, "%ld", &fr[nfr]) == 1)
        nfr++;
    fclose(g);

    rc_tables dflt, tab;
    rc_default_tables(&dflt);
    rc_custom_tables(&tab, &dflt, CUSTOM_STT);

    /* decisions */
    int64_t ndec = 0;
    dec_t d[64];
    static int64_t slotcnt[NCTX][32];
    static int ctxcnt[NCTX];
    for (int64_t i = 0; i < n; i++) {
        int ctx = (uint32_t)sym[i] >> 16;
        int v = (int16_t)(sym[i] & 0xFFFF);
        int m = decisions(v, d);
        ndec += m;
        for (int j = 0; j < m; j++)
            slotcnt[ctx][d[j].slot]++;
        ctxcnt[ctx]++;
    }
    int nctx = 0, topc = 0;
    int64_t topslot = 0;
    for (int c = 0; c < NCTX; c++) {
        if (ctxcnt[c])
            nctx++;
        if (ctxcnt[c] > ctxcnt[topc])
            topc = c;
        for (int k = 0; k < 32; k++)
            if (slotcnt[c][k] > topslot)
                topslot = slotcnt[c][k];
    }
    printf("{\"symbols\": %ld, \"decisions\": %ld, \"decisions_per_symbol\": %.3f, \"contexts_used\": %d, "
           "\"top_context_share\": %.4f, \"top_ctx_slot_share_of_decisions\": %.4f,\n",
           n, ndec, (double)ndec / n, nctx, (double)ctxcnt[topc] / n, (double)topslot / ndec);
    /* cumulative share of the most frequent contexts */
    {
        int *c2 = malloc(sizeof(int) * NCTX);
        memcpy(c2, ctxcnt, sizeof(int) * NCTX);
        qsort(c2, NCTX, sizeof(int), cmp_desc);
        int64_t acc = 0;
        printf(" \"top_k_context_share\": {");
        for (int i = 0, j = 0; i < 256; i++) {
            acc += c2[i];
            if (i + 1 == 4 || i + 1 == 16 || i + 1 == 64 || i + 1 == 128 || i + 1 == 256)
                printf("%s\"%d\": %.4f", j++ ? ", " : "", i + 1, (double)acc / n);
        }
        printf("},\n");
        free(c2);
    }
    /* same-row runs: P(symbol t+1 on symbol t's row) and the symbols a step
     * of up to L same-row symbols covers on average */
    {
        int64_t same = 0;
        for (int64_t i = 1; i < n; i++)
            same += ((uint32_t)sym[i] >> 16) == ((uint32_t)sym[i - 1] >> 16);
        printf(" \"p_same_row\": %.4f, \"symbols_per_run_step\": {", (double)same / (n - 1));
        for (int L = 2; L <= 8; L *= 2) {
            int64_t steps = 0;
            for (int64_t i = 0; i < n;) {
                int64_t j = i + 1;
                while (j < n && j - i < L && ((uint32_t)sym[j] >> 16) == ((uint32_t)sym[i] >> 16))
                    j++;
                steps++;
                i = j;
            }
            printf("%s\"L%d\": %.3f", L > 2 ? ", " : "", L, (double)n / steps);
        }
        printf("},\n");
    }

    /* (a) windows */
    static const int Ws[] = {256, 1024, 4096, 16384, 65536};
    static const int Ps[] = {2, 4, 8, 16};
    printf(" \"windows\": [");
    for (int wi = 0; wi < 5; wi++) {
        int W = Ws[wi];
        double share_sum = 0, share_max = 0, distinct_sum = 0, mk_sum[4] = {0};
        int64_t nw = 0;
        static int cnt[NCTX];
        int *lst = malloc(sizeof(int) * NCTX);
        for (int64_t b = 0; b + W <= n; b += W) {
            memset(cnt, 0, sizeof(cnt));
            for (int64_t i = b; i < b + W; i++)
                cnt[(uint32_t)sym[i] >> 16]++;
            int mx = 0, nd = 0;
            for (int c = 0; c < NCTX; c++)
                if (cnt[c]) {
                    lst[nd++] = cnt[c];
                    if (cnt[c] > mx)
                        mx = cnt[c];
                }
            share_sum += (double)mx / W;
            if ((double)mx / W > share_max)
                share_max = (double)mx / W;
            distinct_sum += nd;
            for (int pi = 0; pi < 4; pi++) {
                int *tmp = malloc(sizeof(int) * nd);
                memcpy(tmp, lst, sizeof(int) * nd);
                mk_sum[pi] += (double)lpt(tmp, nd, Ps[pi]) / ((double)W / Ps[pi]);
                free(tmp);
            }
            nw++;
        }
        free(lst);
        printf("%s{\"W\": %d, \"windows\": %ld, \"top_share_mean\": %.4f, \"top_share_max\": %.4f, "
               "\"contexts_mean\": %.1f, \"makespan_over_ideal\": {\"P2\": %.3f, \"P4\": %.3f, \"P8\": %.3f, "
               "\"P16\": %.3f}}",
               wi ? ",\n   " : "", W, nw, share_sum / nw, share_max, distinct_sum / nw, mk_sum[0] / nw,
               mk_sum[1] / nw, mk_sum[2] / nw, mk_sum[3] / nw);
    }
    printf("],\n");

    /* (b) merging at frame boundaries: true walk, and per boundary the
     * trajectories from wrong starts */
    static uint8_t st[NCTX][32];
    static uint8_t stale[NCTX][32], cur_start[NCTX][32];
    memset(st, 128, sizeof(st));
    memset(stale, 128, sizeof(stale));  /* the keyframe's start: all 128 */
    int64_t pos = 0;
    int64_t dec_fr_total = 0, unmerged_stale = 0, unmerged_all = 0, unmerged_128 = 0;
    int64_t never_all_slots = 0, slots_seen = 0;
    int64_t last_sym_stale_sum = 0, last_sym_all_sum = 0, frames_b = 0;
    for (int fi = 0; fi < nfr; fi++) {
        int64_t fend = pos + fr[fi];
        memcpy(cur_start, st, sizeof(st));
        if (fi >= 1) {
            /* wrong starts: lo/hi sets of all 256 states tracked as a
             * "set of live states" per (ctx, slot) */
            static uint8_t alive[NCTX][32][256];  /* alive[c][k][s]: a start that is still distinct */
            static uint8_t guess_stale[NCTX][32], guess_128[NCTX][32];
            static uint8_t merged_stale[NCTX][32], merged_all[NCTX][32], merged_128[NCTX][32], seen[NCTX][32];
            memset(merged_stale, 0, sizeof(merged_stale));
            memset(merged_all, 0, sizeof(merged_all));
            memset(merged_128, 0, sizeof(merged_128));
            memset(seen, 0, sizeof(seen));
            memcpy(guess_stale, stale, sizeof(stale));
            memset(guess_128, 128, sizeof(guess_128));
            for (int c = 0; c < NCTX; c++)
                if (ctxcnt[c])
                    for (int k = 0; k < 32; k++) {
                        memset(alive[c][k], 0, 256);
                        for (int s = 1; s < 256; s++)
                            alive[c][k][s] = 1; /* state held by some start */
                        merged_stale[c][k] = guess_stale[c][k] == st[c][k];
                        merged_128[c][k] = guess_128[c][k] == st[c][k];
                    }
            int64_t last_stale = pos, last_all = pos;
            uint8_t tmp[256];
            for (int64_t i = pos; i < fend; i++) {
                int ctx = (uint32_t)sym[i] >> 16;
                int v = (int16_t)(sym[i] & 0xFFFF);
                int m = decisions(v, d);
                for (int j = 0; j < m; j++) {
                    int k = d[j].slot, b = d[j].bit;
                    const uint8_t *T = b ? tab.to1 : tab.to0;
                    seen[ctx][k] = 1;
                    dec_fr_total++;
                    if (!merged_stale[ctx][k]) {
                        unmerged_stale++;
                        last_stale = i;
                        guess_stale[ctx][k] = T[guess_stale[ctx][k]];
                    }
                    if (!merged_128[ctx][k]) {
                        unmerged_128++;
                        guess_128[ctx][k] = T[guess_128[ctx][k]];
                    }
                    if (!merged_all[ctx][k]) {
                        unmerged_all++;
                        last_all = i;
                        memset(tmp, 0, 256);
                        int live = 0;
                        for (int s = 1; s < 256; s++)
                            if (alive[ctx][k][s]) {
                                int t2 = T[s];
                                if (!tmp[t2]) {
                                    tmp[t2] = 1;
                                    live++;
                                }
                            }
                        memcpy(alive[ctx][k], tmp, 256);
                        if (live == 1)
                            merged_all[ctx][k] = 1;
                    }
                    st[ctx][k] = T[st[ctx][k]];
                    if (!merged_stale[ctx][k] && guess_stale[ctx][k] == st[ctx][k])
                        merged_stale[ctx][k] = 1;
                    if (!merged_128[ctx][k] && guess_128[ctx][k] == st[ctx][k])
                        merged_128[ctx][k] = 1;
                }
            }
            for (int c = 0; c < NCTX; c++)
                for (int k = 0; k < 32; k++)
                    if (seen[c][k]) {
                        slots_seen++;
                        if (!merged_all[c][k])
                            never_all_slots++;
                    }
            last_sym_stale_sum += last_stale - pos;
            last_sym_all_sum += last_all - pos;
            frames_b++;
        } else {
            for (int64_t i = pos; i < fend; i++) {
                int ctx = (uint32_t)sym[i] >> 16;
                int v = (int16_t)(sym[i] & 0xFFFF);
                int m = decisions(v, d);
                for (int j = 0; j < m; j++) {
                    const uint8_t *T = d[j].bit ? tab.to1 : tab.to0;
                    st[ctx][d[j].slot] = T[st[ctx][d[j].slot]];
                }
            }
        }
        /* the stale guess for boundary fi+1: the true state at the start of frame fi */
        memcpy(stale, cur_start, sizeof(st));
        pos = fend;
    }
    printf(" \"merge\": {\"frame_boundaries\": %ld, \"decisions_in_those_frames\": %ld, "
           "\"unmerged_frac_stale_guess\": %.4f, \"unmerged_frac_guess128\": %.4f, "
           "\"unmerged_frac_all_starts\": %.4f, \"slots_never_coalesced_frac\": %.4f, "
           "\"repair_walk_symbols_frac_stale\": %.4f, \"repair_walk_symbols_frac_all\": %.4f}}\n",
           frames_b, dec_fr_total, (double)unmerged_stale / dec_fr_total, (double)unmerged_128 / dec_fr_total,
           (double)unmerged_all / dec_fr_total, (double)never_all_slots / (slots_seen ? slots_seen : 1),
           (double)last_sym_stale_sum / (frames_b ? frames_b : 1) / ((double)(n - fr[0]) / (nfr - 1)),
           (double)last_sym_all_sum / (frames_b ? frames_b : 1) / ((double)(n - fr[0]) / (nfr - 1)));
    return 0;
}
