// rp_damp.h — flap-damping score arithmetic (lib/membership/member.js:45-66, 133-153), shared by
// the member fold (rp_members.hip) and the decay sweep.
//
// The reference computes the decay factor with JavaScript's Math.pow(Math.E, y). ECMAScript
// leaves Math.pow implementation-approximated; V8 (Node 12.22, the engine the goldens come from)
// implements it as v8::base::ieee754::pow, its port of fdlibm's __ieee754_pow (e_pow.c, Sun
// Microsystems 1993) with one regrouped division in the final reconstruction. That algorithm is
// restated here for x > 0 (the decay passes Math.E) and any y, special cases kept; it reproduced
// Math.pow(Math.E, y) bit for bit on 200,000 decay exponents (tests/golden/damp_golden.json
// carries the engine's own values). Every operation is a
// correctly rounded IEEE double operation: contraction into FMA is switched off, so the result
// does not depend on the compiler or the device. Math.round is restated as V8 lowers it
// (ceil, then step back when ceil - 0.5 > x). The parity plan and its tolerance are in DESIGN.md
// §4.6 and tests/test_damp_gpu.py.
#pragma once

#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

namespace rp {
namespace damp {

struct Config {
    int enabled;           // dampScoringEnabled (config.js:60)
    double initial;        // dampScoringInitial (0)
    double min;            // dampScoringMin (0)
    double max;            // dampScoringMax (10000)
    double penalty;        // dampScoringPenalty (500)
    double suppress;       // dampScoringSuppressLimit (5000)
    double half_life;      // dampScoringHalfLife, seconds (60)
};

__host__ __device__ inline int32_t hi_word(double x) {
    return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}
__host__ __device__ inline uint32_t lo_word(double x) { return (uint32_t)__builtin_bit_cast(uint64_t, x); }
__host__ __device__ inline double from_words(int32_t hi, uint32_t lo) {
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | lo);
}
__host__ __device__ inline double clear_lo(double x) { return from_words(hi_word(x), 0); }

// fdlibm __ieee754_pow for x > 0 finite, x != 1 (the caller passes Math.E) and any y.
__host__ __device__ inline double pow_fdlibm(double x, double y) {
#pragma clang fp contract(off)
    const double two53 = 9007199254740992.0, huge = 1.0e300, tiny = 1.0e-300;
    const double L1 = 5.99999999999994648725e-01, L2 = 4.28571428578550184252e-01,
                 L3 = 3.33333329818377432918e-01, L4 = 2.72728123808534006489e-01,
                 L5 = 2.30660745775561754067e-01, L6 = 2.06975017800338417784e-01;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    const double lg2 = 6.93147180559945286227e-01, lg2_h = 6.93147182464599609375e-01,
                 lg2_l = -1.90465429995776804525e-09, ovt = 8.0085662595372944372e-17;
    const double cp = 9.61796693925975554329e-01, cp_h = 9.61796700954437255859e-01,
                 cp_l = -7.02846165095275826516e-09;
    const double ivln2 = 1.44269504088896338700e+00, ivln2_h = 1.44269502162933349609e+00,
                 ivln2_l = 1.92596299112661746887e-08;
    const double dp_h1 = 5.84962487220764160156e-01, dp_l1 = 1.35003920212974897128e-08;

    const int32_t hx = hi_word(x), hy = hi_word(y);
    const uint32_t ly = lo_word(y);
    int32_t ix = hx & 0x7fffffff;
    const int32_t iy = hy & 0x7fffffff;
    if ((iy | (int32_t)ly) == 0) return 1.0;                     // y == +-0
    if (iy > 0x7ff00000 || (iy == 0x7ff00000 && ly != 0)) return x + y;  // NaN
    if (ly == 0) {
        if (iy == 0x7ff00000) {  // y = +-inf, x > 0, x != 1
            if (ix >= 0x3ff00000) return hy >= 0 ? y : 0.0;
            return hy < 0 ? -y : 0.0;
        }
        if (iy == 0x3ff00000) return hy < 0 ? 1.0 / x : x;
        if (hy == 0x40000000) return x * x;
        if (hy == 0x3fe00000) return std::sqrt(x);
    }
    double ax = x, t1, t2;
    if (iy > 0x41e00000) {  // |y| > 2^31
        if (iy > 0x43f00000) {
            if (ix <= 0x3fefffff) return hy < 0 ? huge * huge : tiny * tiny;
            return hy > 0 ? huge * huge : tiny * tiny;
        }
        if (ix < 0x3fefffff) return hy < 0 ? huge * huge : tiny * tiny;
        if (ix > 0x3ff00000) return hy > 0 ? huge * huge : tiny * tiny;
        const double t = ax - 1.0;
        const double w = (t * t) * (0.5 - t * (0.3333333333333333333333 - t * 0.25));
        const double u = ivln2_h * t;
        const double v = t * ivln2_l - w * ivln2;
        t1 = clear_lo(u + v);
        t2 = v - (t1 - u);
    } else {
        int32_t n = 0;
        if (ix < 0x00100000) {
            ax *= two53;
            n -= 53;
            ix = hi_word(ax);
        }
        n += (ix >> 20) - 0x3ff;
        const int32_t j = ix & 0x000fffff;
        int k;
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
        ax = from_words(ix, lo_word(ax));
        const double bp = k ? 1.5 : 1.0, dp_h = k ? dp_h1 : 0.0, dp_l = k ? dp_l1 : 0.0;
        double u = ax - bp;
        double v = 1.0 / (ax + bp);
        const double ss = u * v;
        const double s_h = clear_lo(ss);
        double t_h = from_words(((ix >> 1) | 0x20000000) + 0x00080000 + (k << 18), 0);
        double t_l = ax - (t_h - bp);
        const double s_l = v * ((u - s_h * t_h) - s_h * t_l);
        double s2 = ss * ss;
        double r = s2 * s2 * (L1 + s2 * (L2 + s2 * (L3 + s2 * (L4 + s2 * (L5 + s2 * L6)))));
        r += s_l * (s_h + ss);
        s2 = s_h * s_h;
        t_h = clear_lo(3.0 + s2 + r);
        t_l = r - ((t_h - 3.0) - s2);
        u = s_h * t_h;
        v = s_l * t_h + t_l * ss;
        const double p_h = clear_lo(u + v);
        const double p_l = v - (p_h - u);
        const double z_h = cp_h * p_h;
        const double z_l = cp_l * p_h + p_l * cp + dp_l;
        const double t = (double)n;
        t1 = clear_lo(((z_h + z_l) + dp_h) + t);
        t2 = z_l - (((t1 - t) - dp_h) - z_h);
    }
    // (y1 + y2) * (t1 + t2)
    const double y1 = clear_lo(y);
    const double p_l = (y - y1) * t1 + y * t2;
    double p_h = y1 * t1;
    double z = p_l + p_h;
    int32_t j = hi_word(z);
    int32_t i = (int32_t)lo_word(z);
    if (j >= 0x40900000) {  // z >= 1024
        if (((j - 0x40900000) | i) != 0 || p_l + ovt > z - p_h) return huge * huge;
    } else if ((j & 0x7fffffff) >= 0x4090cc00) {  // z <= -1075
        if (((j - (int32_t)0xc090cc00) | i) != 0 || p_l <= z - p_h) return tiny * tiny;
    }
    // 2^(p_h + p_l)
    i = j & 0x7fffffff;
    int32_t k = (i >> 20) - 0x3ff;
    int32_t n = 0;
    if (i > 0x3fe00000) {
        n = j + (0x00100000 >> (k + 1));
        k = ((n & 0x7fffffff) >> 20) - 0x3ff;
        const double t = from_words(n & ~(0x000fffff >> k), 0);
        n = ((n & 0x000fffff) | 0x00100000) >> (20 - k);
        if (j < 0) n = -n;
        p_h -= t;
    }
    double t = clear_lo(p_l + p_h);
    const double u = t * lg2_h;
    const double v = (p_l - (t - p_h)) * lg2 + t * lg2_l;
    z = u + v;
    const double w = v - (z - u);
    t = z * z;
    t1 = z - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    // V8's port divides by the whole ((t1 - two) - (w + z * w)) where e_pow.c has
    // (z*t1)/(t1-two) - (w+z*w); this form is the one Math.pow returns
    const double r = (z * t1) / ((t1 - 2.0) - (w + z * w));
    z = 1.0 - (r - z);
    j = hi_word(z) + (n << 20);
    if ((j >> 20) <= 0) return std::ldexp(z, n);  // subnormal result
    return from_words(hi_word(z) + (n << 20), lo_word(z));
}

// Math.round (round half toward +infinity) as V8 lowers it: ceil, then step back.
__host__ __device__ inline double js_round(double x) {
#pragma clang fp contract(off)
    if (!(x == x) || std::isinf(x)) return x;
    double r = std::ceil(x);
    if (r - 0.5 > x) r -= 1.0;
    return r;
}

// decayDampScore (member.js:45-66): the score `last_ts` ms after the last penalty, from the score
// the penalty left (lastUpdateDampScore). A null lastUpdateTimestamp counts as 0, as JS's
// `now - null` does.
__host__ __device__ inline double decayed(const Config& c, double last_score, int64_t last_ts, int64_t now) {
#pragma clang fp contract(off)
    const double since = ((double)now - (double)last_ts) / 1000.0;
    const double decay = pow_fdlibm(2.718281828459045, -1.0 * since * 0.6931471805599453 / c.half_life);
    return std::fmax(js_round(last_score * decay), c.min);
}

// _applyUpdatePenalty (member.js:133-153): decay, add the penalty, clamp to dampScoringMax.
// Returns the new score; *exceeded = the 'suppressLimitExceeded' condition.
__host__ __device__ inline double penalized(const Config& c, double last_score, int64_t last_ts, int64_t now,
                                            bool* exceeded) {
#pragma clang fp contract(off)
    const double s = std::fmin(decayed(c, last_score, last_ts, now) + c.penalty, c.max);
    *exceeded = s > c.suppress;
    return s;
}

}  // namespace damp
}  // namespace rp
