// Host simulation of k_batch_rows' relaxation schedule (scheduling probe,
// not product code): counts vertex processings / arc visits per batch for a
// given bucket width and per-lane bucket offsets, so batch orders and bucket
// rules can be compared on the CPU before a GPU run.
//
// Phase model: candidates = vertices pending at the phase start, processed
// in place (Gauss-Seidel) hubs first then ascending id, like the kernel's
// queue; a vertex's lanes with key = dist - off < bound relax all arcs, the
// other reached lanes keep it pending; the bound advances to the bucket of
// the smallest deferred key only after a phase with no improvement.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    double procs, arcs, phases, lanesAct, cands;
    double touched;     // distinct (vertex, phase) pairs relaxed into (any lane, improving or not)
    double improving;   // arc visits with at least one improving lane
    double laneImp;     // improving lane relaxations
    double skippable;   // arc visits whose head had every lane's key below the last closed
                        // bucket bound (final for all lanes: the D-line read is avoidable)
    double skip2;       // ... and known to be so through a record made when the head was last
                        // processed with all lanes' keys below that phase's bound (2-bitmap scheme)
    double impv;        // distinct vertices improved per phase, summed over phases
    double impvMax;     // ... the largest phase
    double impvOver[4]; // phases with more than 128 / 256 / 512 / 1024 improved vertices
} SimOut;

static const double* g_sortKey;
// hub-cache probe (sim_set_hubs): arc visits / improving visits whose head,
// and vertex processings whose tail, is a marked hub
static const uint8_t* g_hub;
double g_hubArcs, g_hubImp, g_hubProcs;
void sim_set_hubs(const uint8_t* h) { g_hub = h; g_hubArcs = g_hubImp = g_hubProcs = 0; }
void sim_hub_counts(double* o) { o[0] = g_hubArcs; o[1] = g_hubImp; o[2] = g_hubProcs; }
static int cmp_key(const void* a, const void* b) {
    const double x = g_sortKey[*(const int32_t*)a], y = g_sortKey[*(const int32_t*)b];
    return x < y ? -1 : x > y ? 1 : 0;
}

// vkey (optional, [nBatch][n]): a per-VERTEX bucket key replacing every
// lane's dist - off (scheduling experiments: all lanes of a vertex processed
// together at the vertex's key).
int batch_sim(int32_t n, const int32_t* rowPtr, const int32_t* col, const double* lat,
              const int32_t* srcs, const double* offs, int32_t nBatch, int32_t LB, double delta,
              int32_t heavyDeg, int32_t dirtyMode, int32_t farMode, SimOut* out, const double* vkey) {
    double* D = malloc(sizeof(double) * (size_t)n * LB);
    uint8_t* pend = calloc(n, 1);
    uint8_t* nextp = calloc(n, 1);
    int32_t* q = malloc(sizeof(int32_t) * n);
    uint64_t* dirty = calloc(n, 8);
    uint8_t* farp = calloc(n, 1);
    uint8_t* farp2 = calloc(n, 1);   // farMode & 8: keys beyond the next bucket
    int farNext = 0;                 // something entered farp (the next bucket) this bucket
    int32_t* stamp = malloc(sizeof(int32_t) * n);
    int32_t* istamp = malloc(sizeof(int32_t) * n);   // improved in phase gphase
    double* sortKey = malloc(sizeof(double) * n);      // farMode & 16: light-queue order
    uint64_t* hpend = calloc(n, 8);   // lanes whose heavy arcs wait for their bucket to settle
    for (int v = 0; v < n; ++v) stamp[v] = istamp[v] = -1;
    uint8_t* recP = calloc(n, 1);   // all lanes below the bound when last processed (this bucket)
    uint8_t* recF = calloc(n, 1);   // ... in a closed bucket: final
    int32_t gphase = 0;
    if (!D || !pend || !nextp || !q) return -1;
    memset(out, 0, sizeof(*out));
    for (int b = 0; b < nBatch; ++b) {
        const int32_t* s = srcs + (size_t)b * LB;
        const double* off = offs + (size_t)b * LB;
        const double* vk = vkey ? vkey + (size_t)b * n : NULL;
#define KEY(v, l, d) (vk ? vk[v] : (d) - off[l])
#define FARSET(v, k) do { if ((farMode & 8) && (k) >= bound + delta) farp2[v] = 1; \
                          else { farp[v] = 1; farNext = 1; } } while (0)
        for (size_t i = 0; i < (size_t)n * LB; ++i) D[i] = INFINITY;
        memset(pend, 0, n);
        memset(dirty, 0, 8 * (size_t)n);
        memset(farp, 0, n);
        memset(hpend, 0, 8 * (size_t)n);
        memset(recP, 0, n);
        memset(recF, 0, n);
        double farMin = INFINITY;
        double maxOff = 0;
        for (int l = 0; l < LB; ++l) {
            if (s[l] < 0) continue;
            D[(size_t)s[l] * LB + l] = 0.0;
            dirty[s[l]] |= 1ull << l;
            pend[s[l]] = 1;
            if (off[l] > maxOff) maxOff = off[l];
        }
        double closed = -INFINITY;   // keys below it are final
        double bound = -maxOff + delta;
        // start at the bucket of the smallest source key
        {
            double mk = INFINITY;
            for (int l = 0; l < LB; ++l)
                if (s[l] >= 0 && -off[l] < mk) mk = -off[l];
            bound = (floor(mk / delta) + 1.0) * delta;
        }
        for (int guard = 0; guard < 100000; ++guard) {
            int qn = 0;
            for (int v = 0; v < n; ++v)
                if (pend[v] && rowPtr[v + 1] - rowPtr[v] >= heavyDeg) q[qn++] = v;
            const int qh = qn;
            for (int v = 0; v < n; ++v)
                if (pend[v] && rowPtr[v + 1] - rowPtr[v] < heavyDeg) q[qn++] = v;
            if (farMode & 16) {
                // within-phase order: light candidates by their smallest dirty
                // lane key (the order a per-phase key sort would give)
                g_sortKey = sortKey;
                for (int i = qh; i < qn; ++i) {
                    const int v = q[i];
                    double mk = INFINITY;
                    for (int l = 0; l < LB; ++l) {
                        const double d = D[(size_t)v * LB + l];
                        if (d != INFINITY && ((dirty[v] >> l) & 1)) { const double k = KEY(v, l, d); if (k < mk) mk = k; }
                    }
                    sortKey[v] = mk;
                }
                qsort(q + qh, qn - qh, sizeof(int32_t), cmp_key);
            }
            if (qn == 0 && (farMode & 4)) {
                // bucket settled: heavy arcs (w >= delta) of the lanes whose
                // key is below the bound, once, with their final values
                for (int u = 0; u < n; ++u) {
                    if (!hpend[u]) continue;
                    uint64_t go = 0;
                    double du[64];
                    for (int l = 0; l < LB; ++l) {
                        du[l] = D[(size_t)u * LB + l];
                        if (((hpend[u] >> l) & 1) && KEY(u, l, du[l]) < bound) go |= 1ull << l;
                    }
                    if (!go) continue;
                    hpend[u] &= ~go;
                    out->procs += 1;
                    for (int a = rowPtr[u]; a < rowPtr[u + 1]; ++a) {
                        const double w = lat[a];
                        if (w < delta) continue;
                        const int x = col[a];
                        out->arcs += 1;
                        int anyImp = 0;
                        for (int l = 0; l < LB; ++l) {
                            if (!((go >> l) & 1)) continue;
                            const double nb = du[l] + w;
                            if (nb < D[(size_t)x * LB + l]) {
                                D[(size_t)x * LB + l] = nb;
                                const double kx = KEY(x, l, nb);
                                if (kx < bound) nextp[x] = 1;   // cannot happen (w >= delta)
                                else { FARSET(x, kx); if (kx < farMin) farMin = kx; }
                                dirty[x] |= 1ull << l;
                                anyImp = 1;
                                out->laneImp += 1;
                            }
                        }
                        out->improving += anyImp;
                    }
                }
            }
            if (qn == 0) {
                if (!farMode || farMin == INFINITY) break;
                const double mn = farMin;
                farMin = INFINITY;
                double nb = (floor(mn / delta) + 1.0) * delta;
                if (!(mn < nb)) nb = mn + delta;
                closed = bound;
                for (int v = 0; v < n; ++v) if (recP[v]) { recP[v] = 0; recF[v] = 1; }
                bound = nb;
                if (!(farMode & 8)) {
                    memcpy(pend, farp, n);
                    memset(farp, 0, n);
                } else if (farNext) {          // next bucket: near <- F, F <- F2
                    memcpy(pend, farp, n);
                    memcpy(farp, farp2, n);
                    memset(farp2, 0, n);
                } else {                       // jump: near <- F2
                    memcpy(pend, farp2, n);
                    memset(farp, 0, n);
                    memset(farp2, 0, n);
                }
                farNext = 0;
                if (farMode & 8) for (int v = 0; v < n; ++v) if (farp[v]) { farNext = 1; break; }
                continue;
            }
            memset(pend, 0, n);
            memset(nextp, 0, n);
            ++gphase;
            int active = 0;
            int impPhase = 0;
            double minNext = INFINITY;
            out->cands += qn;
            for (int i = 0; i < qn; ++i) {
                const int u = q[i];
                double du[64];
                uint64_t act = 0;
                for (int l = 0; l < LB; ++l) {
                    du[l] = D[(size_t)u * LB + l];
                    if (du[l] == INFINITY) continue;
                    const double key = KEY(u, l, du[l]);
                    if (key < bound) act |= 1ull << l;
                    else if (farMode) {
                        FARSET(u, key);
                        if (key < farMin) farMin = key;
                    } else {
                        nextp[u] = 1;
                        if (key < minNext) minNext = key;
                    }
                }
                if ((farMode & 2) && act) {
                    // eager: every reached lane of u goes with the active ones
                    for (int l = 0; l < LB; ++l)
                        if (du[l] != INFINITY) act |= 1ull << l;
                }
                if (dirtyMode) {
                    uint64_t dm = 0;
                    const uint64_t gmask = dirtyMode >= 64 ? ~0ull : ((1ull << dirtyMode) - 1);
                    for (int g0 = 0; g0 < LB; g0 += dirtyMode)
                        if ((dirty[u] >> g0) & gmask) dm |= gmask << g0;
                    act &= dm;
                }
                if (!act) continue;
                dirty[u] &= ~act;
                out->procs += 1;
                if (g_hub && g_hub[u]) g_hubProcs += 1;
                {
                    int all = 1;
                    for (int l = 0; l < LB; ++l)
                        if (s[l] >= 0 && !(du[l] != INFINITY && KEY(u, l, du[l]) < bound)) all = 0;
                    if (all) recP[u] = 1;
                }
                out->lanesAct += __builtin_popcountll(act);
                if (farMode & 4) hpend[u] |= act;
                for (int a = rowPtr[u]; a < rowPtr[u + 1]; ++a) {
                    const int x = col[a];
                    const double w = lat[a];
                    if ((farMode & 4) && w >= delta) continue;
                    out->arcs += 1;
                    {
                        int all = 1;
                        for (int l = 0; l < LB; ++l) {
                            const double dx = D[(size_t)x * LB + l];
                            if (s[l] >= 0 && !(dx != INFINITY && KEY(x, l, dx) < closed)) all = 0;
                        }
                        out->skippable += all;
                        out->skip2 += recF[x];
                    }
                    if (stamp[x] != gphase) { stamp[x] = gphase; out->touched += 1; }
                    if (g_hub && g_hub[x]) g_hubArcs += 1;
                    int anyImp = 0;
                    for (int l = 0; l < LB; ++l) {
                        if (!((act >> l) & 1)) continue;
                        const double nb = du[l] + w;
                        if (nb < D[(size_t)x * LB + l]) {
                            D[(size_t)x * LB + l] = nb;
                            if (farMode && KEY(x, l, nb) >= bound) {
                                FARSET(x, KEY(x, l, nb));
                                if (KEY(x, l, nb) < farMin) farMin = KEY(x, l, nb);
                            } else {
                                nextp[x] = 1;
                            }
                            dirty[x] |= 1ull << l;
                            if (istamp[x] != gphase) { istamp[x] = gphase; ++impPhase; }
                            active = 1;
                            anyImp = 1;
                            out->laneImp += 1;
                        }
                    }
                    out->improving += anyImp;
                    if (g_hub && g_hub[x]) g_hubImp += anyImp;
                }
            }
            memcpy(pend, nextp, n);
            out->phases += 1;
            out->impv += impPhase;
            if (impPhase > out->impvMax) out->impvMax = impPhase;
            for (int k = 0; k < 4; ++k) out->impvOver[k] += impPhase > (128 << k);
            if (!active && !farMode) {
                const double mn = minNext;
                double nb = (floor(mn / delta) + 1.0) * delta;
                if (!(mn < nb)) nb = mn + delta;
                bound = nb;
            }
        }
    }
    free(D);
    free(pend);
    free(nextp);
    free(q);
    free(dirty);
    free(farp);
    free(farp2);
    free(stamp);
    free(istamp);
    free(sortKey);
    free(hpend);
    free(recP);
    free(recF);
    return 0;
}
