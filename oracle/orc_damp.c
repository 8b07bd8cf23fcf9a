/*
 * orc_damp.c — CPU restatement of ringpop's flap-damping score arithmetic. TEST INFRASTRUCTURE.
 *
 *   Member.decayDampScore        lib/membership/member.js:45-66
 *   Member._applyUpdatePenalty   lib/membership/member.js:133-153
 *   (called from evaluateUpdate  member.js:98-107; decayer index.js:330-383)
 *
 * Math.pow(Math.E, y) is the JS engine's. The goldens come from Node v12.22.9, whose V8
 * implements Math.pow as v8::base::ieee754::pow: fdlibm's __ieee754_pow (e_pow.c, Sun
 * Microsystems 1993) with the final reconstruction's division regrouped as
 * (z*t1) / ((t1-2) - (w+z*w)). orc_js_pow restates that for x > 0; it is checked bit for bit
 * against every (y, Math.pow(Math.E, y)) pair tests/golden/damp_golden.json logged from the
 * reference run. Math.round is restated as V8 lowers it (round half up).
 *
 * Compiled with -ffp-contract=off (oracle/Makefile): each operation is one rounded IEEE
 * double operation, as in the engine.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

static int32_t hiw(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return (int32_t)(u >> 32);
}
static uint32_t low(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return (uint32_t)u;
}
static double mkd(int32_t hi, uint32_t lo) {
    const uint64_t u = ((uint64_t)(uint32_t)hi << 32) | lo;
    double d;
    memcpy(&d, &u, 8);
    return d;
}
static double lo0(double x) { return mkd(hiw(x), 0); }

double orc_js_pow(double x, double y) {
    static const double bp[2] = {1.0, 1.5};
    static const double dp_h[2] = {0.0, 5.84962487220764160156e-01}; /* 0x3FE2B803 40000000 */
    static const double dp_l[2] = {0.0, 1.35003920212974897128e-08}; /* 0x3E4CFDEB 43CFD006 */
    static const double two53 = 9007199254740992.0, huge = 1.0e300, tiny = 1.0e-300;
    /* (3/2)(log(x) - 2s - 2/3 s^3) polynomial */
    static const double L1 = 5.99999999999994648725e-01, L2 = 4.28571428578550184252e-01,
                        L3 = 3.33333329818377432918e-01, L4 = 2.72728123808534006489e-01,
                        L5 = 2.30660745775561754067e-01, L6 = 2.06975017800338417784e-01;
    /* exp remez polynomial */
    static const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                        P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                        P5 = 4.13813679705723846039e-08;
    static const double lg2 = 6.93147180559945286227e-01, lg2_h = 6.93147182464599609375e-01,
                        lg2_l = -1.90465429995776804525e-09, ovt = 8.0085662595372944372e-17;
    static const double cp = 9.61796693925975554329e-01, cp_h = 9.61796700954437255859e-01,
                        cp_l = -7.02846165095275826516e-09; /* 2/(3 ln 2) */
    static const double ivln2 = 1.44269504088896338700e+00, ivln2_h = 1.44269502162933349609e+00,
                        ivln2_l = 1.92596299112661746887e-08;
    double z, ax, z_h, z_l, p_h, p_l, y1, t1, t2, r, t, u, v, w;
    int32_t i, j, k, n, hx, hy, ix, iy;
    uint32_t ly;

    hx = hiw(x);
    hy = hiw(y);
    ly = low(y);
    ix = hx & 0x7fffffff;
    iy = hy & 0x7fffffff;
    if ((iy | (int32_t)ly) == 0) return 1.0;
    if (iy > 0x7ff00000 || (iy == 0x7ff00000 && ly != 0)) return x + y;
    if (ly == 0) {
        if (iy == 0x7ff00000) return ix >= 0x3ff00000 ? (hy >= 0 ? y : 0.0) : (hy < 0 ? -y : 0.0);
        if (iy == 0x3ff00000) return hy < 0 ? 1.0 / x : x;
        if (hy == 0x40000000) return x * x;
        if (hy == 0x3fe00000) return sqrt(x);
    }
    ax = x;
    if (iy > 0x41e00000) { /* |y| > 2^31 */
        if (iy > 0x43f00000) return (ix <= 0x3fefffff) == (hy < 0) ? huge * huge : tiny * tiny;
        if (ix < 0x3fefffff) return hy < 0 ? huge * huge : tiny * tiny;
        if (ix > 0x3ff00000) return hy > 0 ? huge * huge : tiny * tiny;
        t = ax - 1.0;
        w = (t * t) * (0.5 - t * (0.3333333333333333333333 - t * 0.25));
        u = ivln2_h * t;
        v = t * ivln2_l - w * ivln2;
        t1 = lo0(u + v);
        t2 = v - (t1 - u);
    } else {
        double ss, s2, s_h, s_l, t_h, t_l;
        n = 0;
        if (ix < 0x00100000) {
            ax *= two53;
            n -= 53;
            ix = hiw(ax);
        }
        n += (ix >> 20) - 0x3ff;
        j = ix & 0x000fffff;
        ix = j | 0x3ff00000;
        if (j <= 0x3988E) {
            k = 0;
        } else if (j < 0xBB67A) {
            k = 1;
        } else {
            k = 0;
            n += 1;
            ix -= 0x00100000;
        }
        ax = mkd(ix, low(ax));
        u = ax - bp[k];
        v = 1.0 / (ax + bp[k]);
        ss = u * v;
        s_h = lo0(ss);
        t_h = mkd(((ix >> 1) | 0x20000000) + 0x00080000 + (k << 18), 0);
        t_l = ax - (t_h - bp[k]);
        s_l = v * ((u - s_h * t_h) - s_h * t_l);
        s2 = ss * ss;
        r = s2 * s2 * (L1 + s2 * (L2 + s2 * (L3 + s2 * (L4 + s2 * (L5 + s2 * L6)))));
        r += s_l * (s_h + ss);
        s2 = s_h * s_h;
        t_h = lo0(3.0 + s2 + r);
        t_l = r - ((t_h - 3.0) - s2);
        u = s_h * t_h;
        v = s_l * t_h + t_l * ss;
        p_h = lo0(u + v);
        p_l = v - (p_h - u);
        z_h = cp_h * p_h;
        z_l = cp_l * p_h + p_l * cp + dp_l[k];
        t = (double)n;
        t1 = lo0(((z_h + z_l) + dp_h[k]) + t);
        t2 = z_l - (((t1 - t) - dp_h[k]) - z_h);
    }
    y1 = lo0(y);
    p_l = (y - y1) * t1 + y * t2;
    p_h = y1 * t1;
    z = p_l + p_h;
    j = hiw(z);
    i = (int32_t)low(z);
    if (j >= 0x40900000) {
        if (((j - 0x40900000) | i) != 0) return huge * huge;
        if (p_l + ovt > z - p_h) return huge * huge;
    } else if ((j & 0x7fffffff) >= 0x4090cc00) {
        if (((j - (int32_t)0xc090cc00) | i) != 0) return tiny * tiny;
        if (p_l <= z - p_h) return tiny * tiny;
    }
    i = j & 0x7fffffff;
    k = (i >> 20) - 0x3ff;
    n = 0;
    if (i > 0x3fe00000) {
        n = j + (0x00100000 >> (k + 1));
        k = ((n & 0x7fffffff) >> 20) - 0x3ff;
        t = mkd(n & ~(0x000fffff >> k), 0);
        n = ((n & 0x000fffff) | 0x00100000) >> (20 - k);
        if (j < 0) n = -n;
        p_h -= t;
    }
    t = lo0(p_l + p_h);
    u = t * lg2_h;
    v = (p_l - (t - p_h)) * lg2 + t * lg2_l;
    z = u + v;
    w = v - (z - u);
    t = z * z;
    t1 = z - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    r = (z * t1) / ((t1 - 2.0) - (w + z * w)); /* V8's grouping (see header) */
    z = 1.0 - (r - z);
    j = hiw(z) + (n << 20);
    if ((j >> 20) <= 0) return scalbn(z, n);
    return mkd(hiw(z) + (n << 20), low(z));
}

/* Math.round: half up, as V8 lowers it (ceil, step back when ceil - 0.5 > x). */
double orc_js_round(double x) {
    if (isnan(x) || isinf(x)) return x;
    double r = ceil(x);
    if (r - 0.5 > x) r -= 1.0;
    return r;
}

/* decayDampScore (member.js:45-66); last_ts 0 = null lastUpdateTimestamp. */
double orc_damp_decayed(const orc_damp_cfg *c, double last_score, int64_t last_ts, int64_t now) {
    const double since = ((double)now - (double)last_ts) / 1000.0;                          /* :55 */
    const double decay = orc_js_pow(2.718281828459045, -1 * since * 0.6931471805599453 / c->half_life); /* :56-57 */
    const double s = orc_js_round(last_score * decay);                                     /* :62-63 */
    return s > c->min ? s : c->min;  /* Math.max(s, min) for non-NaN s */
}

/* _applyUpdatePenalty (member.js:133-153): returns the new score, *exceeded = score > limit. */
double orc_damp_penalized(const orc_damp_cfg *c, double last_score, int64_t last_ts, int64_t now, int *exceeded) {
    double s = orc_damp_decayed(c, last_score, last_ts, now) + c->penalty; /* :136-139 */
    if (s > c->max) s = c->max;
    *exceeded = s > c->suppress_limit; /* :141-142 */
    return s;
}

/* The decayer over n members (index.js:374-383): score[i] for every present member. */
void orc_damp_decay_all(const orc_damp_cfg *c, const uint8_t *exists, const double *last_score,
                        const int64_t *last_ts, uint32_t n, int64_t now, double *score) {
    for (uint32_t i = 0; i < n; i++)
        if (exists[i]) score[i] = orc_damp_decayed(c, last_score[i], last_ts[i], now);
}
