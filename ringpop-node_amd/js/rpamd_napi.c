/*
 * rpamd_napi.c — Node N-API addon over librpamd.so (include/ringpop_amd.h).
 *
 * This is the "thin Node N-API C-ABI addon calling HIP" of BASELINE.json north_star: it
 * only marshals JS values into the C ABI's plain buffers; every hash, sort, lookup, merge and
 * gossip round runs in librpamd's HIP kernels. There is no JS or CPU fallback — a missing
 * library or device raises. The JS classes that mirror the reference's API (lib/ring/index.js
 * HashRing, Membership.update, farmhash.hash32) are in index.js next to this file.
 *
 * Built by ./Makefile (gcc, N-API v3+ headers of the node in this image, rpath to ..).
 */
#include <node_api.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ringpop_amd.h"

/* ------------------------------------------------------------------ helpers */
#define NAPI_OK(call)                                                                 \
    do {                                                                              \
        if ((call) != napi_ok) {                                                      \
            const napi_extended_error_info *ei_ = NULL;                               \
            napi_get_last_error_info(env, &ei_);                                      \
            napi_throw_error(env, NULL, ei_ && ei_->error_message ? ei_->error_message \
                                                                  : "napi call failed"); \
            return NULL;                                                              \
        }                                                                             \
    } while (0)

#define RP_OK(call)                                                \
    do {                                                           \
        if ((call) != 0) {                                         \
            napi_throw_error(env, "ERR_RINGPOP_AMD", rp_last_error()); \
            return NULL;                                           \
        }                                                          \
    } while (0)

#define ARGS(N)                                                            \
    size_t argc = (N);                                                     \
    napi_value argv[(N) > 0 ? (N) : 1];                                    \
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, NULL, NULL));         \
    if (argc < (N)) {                                                      \
        napi_throw_type_error(env, NULL, "wrong number of arguments");     \
        return NULL;                                                       \
    }

static int64_t *f64_to_i64(napi_env env, const double *d, size_t n, int nan_is_min, const char *what);

static napi_value make_u32(napi_env env, uint32_t v) {
    napi_value out;
    napi_create_uint32(env, v, &out);
    return out;
}

static napi_value make_bool(napi_env env, int v) {
    napi_value out;
    napi_get_boolean(env, v != 0, &out);
    return out;
}

static napi_value make_null(napi_env env) {
    napi_value out;
    napi_get_null(env, &out);
    return out;
}

static int is_nullish(napi_env env, napi_value v) {
    napi_valuetype t;
    if (napi_typeof(env, v, &t) != napi_ok) return 1;
    return t == napi_null || t == napi_undefined;
}

/* Handles are napi externals whose finalizer destroys the native object unless destroy()
 * already did (the slot is then NULL). */
typedef struct {
    int kind; /* 1 ring, 2 members, 3 sim */
    void *p;
} handle_t;

static void handle_finalize(napi_env env, void *data, void *hint) {
    (void)env;
    (void)hint;
    handle_t *h = (handle_t *)data;
    if (h->p) {
        if (h->kind == 1) rp_ring_destroy((rp_ring *)h->p);
        if (h->kind == 2) rp_members_destroy((rp_members *)h->p);
        if (h->kind == 3) rp_sim_destroy((rp_sim *)h->p);
    }
    free(h);
}

static napi_value wrap_handle(napi_env env, int kind, void *p) {
    handle_t *h = (handle_t *)malloc(sizeof(handle_t));
    h->kind = kind;
    h->p = p;
    napi_value out;
    if (napi_create_external(env, h, handle_finalize, NULL, &out) != napi_ok) {
        handle_finalize(env, h, NULL);
        napi_throw_error(env, NULL, "napi_create_external failed");
        return NULL;
    }
    return out;
}

static handle_t *get_handle(napi_env env, napi_value v, int kind) {
    void *data = NULL;
    if (napi_get_value_external(env, v, &data) != napi_ok || !data ||
        ((handle_t *)data)->kind != kind) {
        napi_throw_type_error(env, NULL, "invalid ringpop_amd handle");
        return NULL;
    }
    if (!((handle_t *)data)->p) {
        napi_throw_error(env, NULL, "ringpop_amd handle already destroyed");
        return NULL;
    }
    return (handle_t *)data;
}

/* A JS array of strings packed as bytes + offsets (off32 or off64 chosen by the caller). */
typedef struct {
    char *bytes;
    uint32_t *off32;
    uint64_t *off64;
    uint32_t n;
} strpack_t;

static void strpack_free(strpack_t *s) {
    free(s->bytes);
    free(s->off32);
    free(s->off64);
    memset(s, 0, sizeof(*s));
}

/* Returns 0 and fills *s, or -1 with a pending JS exception. Non-strings are coerced with
 * String(x), as the reference's hashFunc(str) would (farmhash takes its argument's string). */
static int strpack_from_array(napi_env env, napi_value arr, strpack_t *s) {
    memset(s, 0, sizeof(*s));
    if (is_nullish(env, arr)) return 0;
    bool isarr = false;
    napi_is_array(env, arr, &isarr);
    if (!isarr) {
        napi_throw_type_error(env, NULL, "expected an array of strings");
        return -1;
    }
    uint32_t n = 0;
    napi_get_array_length(env, arr, &n);
    s->n = n;
    s->off32 = (uint32_t *)malloc(sizeof(uint32_t) * (n + 1));
    s->off64 = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    size_t cap = 64 + (size_t)n * 40, used = 0;
    s->bytes = (char *)malloc(cap);
    for (uint32_t i = 0; i < n; i++) {
        napi_value e, str;
        napi_get_element(env, arr, i, &e);
        if (napi_coerce_to_string(env, e, &str) != napi_ok) {
            strpack_free(s);
            napi_throw_type_error(env, NULL, "array element is not coercible to string");
            return -1;
        }
        size_t len = 0;
        napi_get_value_string_utf8(env, str, NULL, 0, &len);
        if (used + len + 1 > cap) {
            while (used + len + 1 > cap) cap *= 2;
            s->bytes = (char *)realloc(s->bytes, cap);
        }
        size_t got = 0;
        napi_get_value_string_utf8(env, str, s->bytes + used, len + 1, &got);
        s->off32[i] = (uint32_t)used;
        s->off64[i] = used;
        used += got;
    }
    s->off32[n] = (uint32_t)used;
    s->off64[n] = used;
    return 0;
}

/* Typed-array view of the wanted element type: 0 with data/len, or -1 (data NULL, len 0)
 * when v is not such a typed array. Zero-length arrays may have data == NULL. */
static int typed_get(napi_env env, napi_value v, napi_typedarray_type want, void **data, size_t *len) {
    bool is = false;
    *data = NULL;
    *len = 0;
    if (napi_is_typedarray(env, v, &is) != napi_ok || !is) return -1;
    napi_typedarray_type t;
    napi_value ab;
    size_t boff = 0;
    napi_get_typedarray_info(env, v, &t, len, data, &ab, &boff);
    if (t != want) {
        *data = NULL;
        *len = 0;
        return -1;
    }
    return 0;
}

static void *typed_data(napi_env env, napi_value v, napi_typedarray_type want, size_t *len) {
    void *d = NULL;
    typed_get(env, v, want, &d, len);
    return d;
}

static napi_value new_typed(napi_env env, napi_typedarray_type t, size_t n, size_t elem, void **data) {
    napi_value ab, out;
    if (napi_create_arraybuffer(env, n * elem, data, &ab) != napi_ok) return NULL;
    if (napi_create_typedarray(env, t, n, ab, 0, &out) != napi_ok) return NULL;
    return out;
}

static napi_value ring_name(napi_env env, rp_ring *r, uint32_t id) {
    if (id == RP_NULL_ID) return make_null(env);
    uint32_t len = 0;
    const char *p = rp_ring_owner_name(r, id, &len);
    if (!p) return make_null(env);
    napi_value s;
    napi_create_string_utf8(env, p, len, &s);
    return s;
}

/* ------------------------------------------------------------------ common */
static napi_value js_version(napi_env env, napi_callback_info info) {
    (void)info;
    return make_u32(env, rp_version());
}

static napi_value js_device_count(napi_env env, napi_callback_info info) {
    (void)info;
    int n = 0;
    RP_OK(rp_device_count(&n));
    return make_u32(env, (uint32_t)n);
}

/* farmhash.hash32(str) (reference package.json:34): host C++ farmhashmk::Hash32 of the UTF-8
 * bytes, the same code librpamd's kernels run. */
static napi_value js_hash32(napi_env env, napi_callback_info info) {
    ARGS(1);
    napi_value str;
    NAPI_OK(napi_coerce_to_string(env, argv[0], &str));
    size_t len = 0;
    NAPI_OK(napi_get_value_string_utf8(env, str, NULL, 0, &len));
    char stackbuf[256];
    char *buf = len < sizeof(stackbuf) ? stackbuf : (char *)malloc(len + 1);
    napi_get_value_string_utf8(env, str, buf, len + 1, &len);
    uint32_t h = rp_hash32(buf, len);
    if (buf != stackbuf) free(buf);
    return make_u32(env, h);
}

/* ------------------------------------------------------------------ ring */
static napi_value js_ring_create(napi_env env, napi_callback_info info) {
    ARGS(2);
    uint32_t rp = 0;
    int32_t dev = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[0], &rp));
    NAPI_OK(napi_get_value_int32(env, argv[1], &dev));
    rp_ring *r = NULL;
    RP_OK(rp_ring_create(rp, dev, &r));
    return wrap_handle(env, 1, r);
}

static napi_value js_destroy(napi_env env, napi_callback_info info) {
    ARGS(1);
    void *data = NULL;
    NAPI_OK(napi_get_value_external(env, argv[0], &data));
    handle_t *h = (handle_t *)data;
    if (h && h->p) {
        if (h->kind == 1) rp_ring_destroy((rp_ring *)h->p);
        if (h->kind == 2) rp_members_destroy((rp_members *)h->p);
        if (h->kind == 3) rp_sim_destroy((rp_sim *)h->p);
        h->p = NULL;
    }
    return NULL;
}

/* addRemoveServers(add[], remove[], addTokens?, removeTokens?) -> ringChanged
 * (lib/ring/index.js:60-94). Token arrays (Uint32Array, n*replicaPoints) carry a caller
 * hashFunc's replica hashes (options.hashFunc, :29). */
static napi_value js_ring_add_remove(napi_env env, napi_callback_info info) {
    ARGS(5);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    strpack_t add, rem;
    if (strpack_from_array(env, argv[1], &add)) return NULL;
    if (strpack_from_array(env, argv[2], &rem)) {
        strpack_free(&add);
        return NULL;
    }
    size_t n1 = 0, n2 = 0;
    const uint32_t *at = is_nullish(env, argv[3]) ? NULL : (const uint32_t *)typed_data(env, argv[3], napi_uint32_array, &n1);
    const uint32_t *rt = is_nullish(env, argv[4]) ? NULL : (const uint32_t *)typed_data(env, argv[4], napi_uint32_array, &n2);
    int changed = 0;
    int rc = rp_ring_add_remove((rp_ring *)h->p, add.bytes, add.off32, add.n, at, rem.bytes, rem.off32, rem.n, rt,
                                &changed);
    strpack_free(&add);
    strpack_free(&rem);
    RP_OK(rc);
    return make_bool(env, changed);
}

static napi_value js_ring_checksum(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint32_t v = 0;
    int set = 0;
    RP_OK(rp_ring_checksum((rp_ring *)h->p, &v, &set));
    return set ? make_u32(env, v) : make_null(env);
}

static napi_value js_ring_checksum_string(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint64_t len = 0;
    RP_OK(rp_ring_checksum_string((rp_ring *)h->p, NULL, 0, &len));
    char *buf = (char *)malloc(len + 1);
    int rc = rp_ring_checksum_string((rp_ring *)h->p, buf, len, &len);
    if (rc) {
        free(buf);
        RP_OK(rc);
    }
    napi_value s;
    napi_create_string_utf8(env, buf, len, &s);
    free(buf);
    return s;
}

static napi_value js_ring_server_count(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint32_t n = 0;
    RP_OK(rp_ring_server_count((rp_ring *)h->p, &n));
    return make_u32(env, n);
}

static napi_value js_ring_service(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint32_t idle = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &idle));
    RP_OK(rp_ring_service((rp_ring *)h->p, idle));
    return make_u32(env, idle);
}

static napi_value js_ring_token_count(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint32_t n = 0;
    RP_OK(rp_ring_token_count((rp_ring *)h->p, &n));
    return make_u32(env, n);
}

static napi_value js_ring_has_server(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    napi_value str;
    NAPI_OK(napi_coerce_to_string(env, argv[1], &str));
    size_t len = 0;
    napi_get_value_string_utf8(env, str, NULL, 0, &len);
    char *buf = (char *)malloc(len + 1);
    napi_get_value_string_utf8(env, str, buf, len + 1, &len);
    int has = 0;
    int rc = rp_ring_has_server((rp_ring *)h->p, buf, (uint32_t)len, &has);
    free(buf);
    RP_OK(rc);
    return make_bool(env, has);
}

/* Object.keys(servers) in insertion order (getStats, lib/ring/index.js:111-116). */
static napi_value js_ring_servers(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    uint32_t n = 0;
    RP_OK(rp_ring_servers(r, NULL, 0, &n));
    uint32_t *ids = (uint32_t *)malloc(sizeof(uint32_t) * (n ? n : 1));
    int rc = rp_ring_servers(r, ids, n, &n);
    if (rc) {
        free(ids);
        RP_OK(rc);
    }
    napi_value arr;
    napi_create_array_with_length(env, n, &arr);
    for (uint32_t i = 0; i < n; i++) napi_set_element(env, arr, i, ring_name(env, r, ids[i]));
    free(ids);
    return arr;
}

static napi_value js_ring_owner_name(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    uint32_t id = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &id));
    return ring_name(env, (rp_ring *)h->p, id);
}

/* lookupBatch(h, keys[]) -> names (null for an empty ring), lookup() of every key
 * (lib/ring/index.js:145-154), one device launch. */
static napi_value js_ring_lookup(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    strpack_t keys;
    if (strpack_from_array(env, argv[1], &keys)) return NULL;
    uint32_t *own = (uint32_t *)malloc(sizeof(uint32_t) * (keys.n ? keys.n : 1));
    int rc = rp_ring_lookup(r, keys.bytes, keys.off64, 0, keys.n, own);
    uint32_t n = keys.n;
    strpack_free(&keys);
    if (rc) {
        free(own);
        RP_OK(rc);
    }
    napi_value arr;
    napi_create_array_with_length(env, n, &arr);
    for (uint32_t i = 0; i < n; i++) napi_set_element(env, arr, i, ring_name(env, r, own[i]));
    free(own);
    return arr;
}

/* lookup1(h, key) -> name | null and lookupN1(h, key, n) -> [names]: one key, no arrays in
 * between (RingPop.lookup / lookupN per request, index.js:434-471; the ring service, when on,
 * answers them without a launch). */
static int key_utf8(napi_env env, napi_value v, char *stack, size_t cap, char **out, size_t *len) {
    napi_value str;
    if (napi_coerce_to_string(env, v, &str) != napi_ok) {
        napi_throw_type_error(env, NULL, "key is not coercible to string");
        return -1;
    }
    napi_get_value_string_utf8(env, str, NULL, 0, len);
    *out = *len < cap ? stack : (char *)malloc(*len + 1);
    size_t got = 0;
    napi_get_value_string_utf8(env, str, *out, *len + 1, &got);
    *len = got;
    return 0;
}

static napi_value js_ring_lookup1(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    char stack[256], *k = NULL;
    size_t len = 0;
    if (key_utf8(env, argv[1], stack, sizeof stack, &k, &len)) return NULL;
    uint64_t off[2] = {0, len};
    uint32_t own = RP_NULL_ID;
    int rc = rp_ring_lookup(r, k, off, 0, 1, &own);
    if (k != stack) free(k);
    RP_OK(rc);
    return ring_name(env, r, own);
}

static napi_value js_ring_lookupn1(napi_env env, napi_callback_info info) {
    ARGS(3);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    int32_t nrep = 0;
    NAPI_OK(napi_get_value_int32(env, argv[2], &nrep));
    char stack[256], *k = NULL;
    size_t len = 0;
    if (key_utf8(env, argv[1], stack, sizeof stack, &k, &len)) return NULL;
    const uint32_t W = nrep > 1 ? (uint32_t)nrep : 1u;
    uint32_t own_s[16], *own = W <= 16 ? own_s : (uint32_t *)malloc(4ull * W);
    uint8_t cnt = 0;
    uint64_t off[2] = {0, len};
    int rc = rp_ring_lookupn(r, k, off, 0, 1, nrep, own, &cnt);
    if (k != stack) free(k);
    if (rc) {
        if (own != own_s) free(own);
        RP_OK(rc);
    }
    napi_value arr;
    napi_create_array_with_length(env, cnt, &arr);
    for (uint32_t j = 0; j < cnt; j++) napi_set_element(env, arr, j, ring_name(env, r, own[j]));
    if (own != own_s) free(own);
    return arr;
}

/* groupKeys(h, keys[] | Uint32Array hashes) -> {dests: [name|null], groupOff: Uint32Array,
 * perm: Uint32Array}: handleOrProxyAll's _.groupBy(keys, lookup) (index.js:609-667, :616) and
 * lookupKeys (lib/request-proxy/send.js:171-179) on the device. A null dest = the empty ring's
 * null owner (the caller substitutes whoami(), index.js:434-451). */
static napi_value js_ring_group_keys(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    bool is_typed = false;
    napi_is_typedarray(env, argv[1], &is_typed);
    size_t n = 0;
    void *hv = NULL;
    strpack_t keys;
    memset(&keys, 0, sizeof(keys));
    if (is_typed) {
        if (typed_get(env, argv[1], napi_uint32_array, &hv, &n)) {
            napi_throw_type_error(env, NULL, "hashes must be a Uint32Array");
            return NULL;
        }
    } else {
        if (strpack_from_array(env, argv[1], &keys)) return NULL;
        n = keys.n;
    }
    size_t nn = n ? n : 1;
    uint32_t *dests = (uint32_t *)malloc(sizeof(uint32_t) * nn);
    void *gd = NULL, *pd = NULL;
    napi_value goff = new_typed(env, napi_uint32_array, nn + 1, 4, &gd);
    napi_value perm = new_typed(env, napi_uint32_array, n, 4, &pd);
    uint32_t nd = 0;
    uint32_t pdummy = 0;
    int rc = is_typed ? rp_ring_group_hashes(r, (const uint32_t *)hv, n, RP_NULL_ID, dests, (uint32_t *)gd,
                                             n ? (uint32_t *)pd : &pdummy, &nd)
                      : rp_ring_group_keys(r, keys.bytes, keys.off64, 0, n, RP_NULL_ID, dests, (uint32_t *)gd,
                                           n ? (uint32_t *)pd : &pdummy, &nd);
    if (!is_typed) strpack_free(&keys);
    if (rc) {
        free(dests);
        RP_OK(rc);
    }
    napi_value arr, out;
    napi_create_array_with_length(env, nd, &arr);
    for (uint32_t i = 0; i < nd; i++) napi_set_element(env, arr, i, ring_name(env, r, dests[i]));
    free(dests);
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "dests", arr);
    napi_set_named_property(env, out, "groupOff", goff);
    napi_set_named_property(env, out, "perm", perm);
    return out;
}

/* lookupNBatch(h, keys[], n) -> arrays of names, lookupN() of every key (:157-189). */
static napi_value js_ring_lookupn(napi_env env, napi_callback_info info) {
    ARGS(3);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    rp_ring *r = (rp_ring *)h->p;
    int32_t nrep = 0;
    NAPI_OK(napi_get_value_int32(env, argv[2], &nrep));
    strpack_t keys;
    if (strpack_from_array(env, argv[1], &keys)) return NULL;
    uint32_t w = nrep > 1 ? (uint32_t)nrep : 1u;
    uint32_t n = keys.n;
    uint32_t *own = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n ? n : 1) * w);
    uint8_t *cnt = (uint8_t *)malloc(n ? n : 1);
    int rc = rp_ring_lookupn(r, keys.bytes, keys.off64, 0, n, nrep, own, cnt);
    strpack_free(&keys);
    if (rc) {
        free(own);
        free(cnt);
        RP_OK(rc);
    }
    napi_value arr;
    napi_create_array_with_length(env, n, &arr);
    for (uint32_t i = 0; i < n; i++) {
        napi_value row;
        napi_create_array_with_length(env, cnt[i], &row);
        for (uint32_t j = 0; j < cnt[i]; j++)
            napi_set_element(env, row, j, ring_name(env, r, own[(size_t)i * w + j]));
        napi_set_element(env, arr, i, row);
    }
    free(own);
    free(cnt);
    return arr;
}

/* lookupNHashes(h, Uint32Array hashes, n) -> {owners: Uint32Array(ids), counts: Uint8Array}:
 * the id-level batch for callers with their own hashFunc or that keep owner ids. */
static napi_value js_ring_lookupn_hashes(napi_env env, napi_callback_info info) {
    ARGS(3);
    handle_t *h = get_handle(env, argv[0], 1);
    if (!h) return NULL;
    size_t n = 0;
    void *hv = NULL;
    if (typed_get(env, argv[1], napi_uint32_array, &hv, &n)) {
        napi_throw_type_error(env, NULL, "hashes must be a Uint32Array");
        return NULL;
    }
    const uint32_t *hs = (const uint32_t *)hv;
    int32_t nrep = 0;
    NAPI_OK(napi_get_value_int32(env, argv[2], &nrep));
    size_t w = nrep > 1 ? (size_t)nrep : 1;
    void *od = NULL, *cd = NULL;
    napi_value owners = new_typed(env, napi_uint32_array, n * w, 4, &od);
    napi_value counts = new_typed(env, napi_uint8_array, n, 1, &cd);
    if (!owners || !counts) {
        napi_throw_error(env, NULL, "allocation failed");
        return NULL;
    }
    if (n) RP_OK(rp_ring_lookupn_hashes((rp_ring *)h->p, hs, n, nrep, (uint32_t *)od, (uint8_t *)cd));
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "owners", owners);
    napi_set_named_property(env, out, "counts", counts);
    return out;
}

/* ------------------------------------------------------------------ membership */
static napi_value js_members_create(napi_env env, napi_callback_info info) {
    ARGS(2);
    uint32_t cap = 0;
    int32_t dev = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[0], &cap));
    NAPI_OK(napi_get_value_int32(env, argv[1], &dev));
    rp_members *m = NULL;
    RP_OK(rp_members_create(cap, dev, &m));
    return wrap_handle(env, 2, m);
}

static napi_value js_members_intern(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    strpack_t s;
    if (strpack_from_array(env, argv[1], &s)) return NULL;
    void *d = NULL;
    napi_value ids = new_typed(env, napi_uint32_array, s.n, 4, &d);
    int rc = s.n ? rp_members_intern((rp_members *)h->p, s.bytes, s.off32, s.n, (uint32_t *)d) : 0;
    strpack_free(&s);
    RP_OK(rc);
    return ids;
}

static napi_value js_members_set_local(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    uint32_t id = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &id));
    RP_OK(rp_members_set_local((rp_members *)h->p, id));
    return NULL;
}

/* update(h, ids Uint32Array, status Uint8Array, inc Float64Array, nowMs) ->
 * {applied: Uint8Array, status: Uint8Array, inc: Float64Array, nApplied} — Membership.update
 * (lib/membership/index.js:249-324) over evaluateUpdate (member.js:71-202). Incarnation
 * numbers are JS Numbers (Date.now() values), exact as doubles. */
static napi_value js_members_update(napi_env env, napi_callback_info info) {
    ARGS(5);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    size_t k = 0, k2 = 0, k3 = 0;
    const uint32_t *ids = (const uint32_t *)typed_data(env, argv[1], napi_uint32_array, &k);
    const uint8_t *st = (const uint8_t *)typed_data(env, argv[2], napi_uint8_array, &k2);
    const double *incd = (const double *)typed_data(env, argv[3], napi_float64_array, &k3);
    if ((k && (!ids || !st || !incd)) || k2 != k || k3 != k) {
        napi_throw_type_error(env, NULL, "update expects Uint32Array ids, Uint8Array status, Float64Array inc of equal length");
        return NULL;
    }
    double now = 0;
    NAPI_OK(napi_get_value_double(env, argv[4], &now));
    int64_t now64 = 0;
    {
        int64_t *t = f64_to_i64(env, &now, 1, 0, "update: now");
        if (!t) return NULL;
        now64 = t[0];
        free(t);
    }
    int64_t *inc = f64_to_i64(env, incd, k, 0, "update: incarnationNumber");
    if (!inc) return NULL;
    void *ad = NULL, *sd = NULL, *id = NULL;
    napi_value applied = new_typed(env, napi_uint8_array, k, 1, &ad);
    napi_value nst = new_typed(env, napi_uint8_array, k, 1, &sd);
    napi_value ninc = new_typed(env, napi_float64_array, k, 8, &id);
    int64_t *ninc64 = (int64_t *)malloc(sizeof(int64_t) * (k ? k : 1));
    uint32_t napplied = 0;
    int rc = k ? rp_members_update((rp_members *)h->p, ids, st, inc, (uint32_t)k, now64, (uint8_t *)ad,
                                   (uint8_t *)sd, ninc64, &napplied)
               : 0;
    for (size_t i = 0; rc == 0 && i < k; i++) ((double *)id)[i] = (double)ninc64[i];
    free(inc);
    free(ninc64);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "applied", applied);
    napi_set_named_property(env, out, "status", nst);
    napi_set_named_property(env, out, "inc", ninc);
    napi_set_named_property(env, out, "nApplied", make_u32(env, napplied));
    return out;
}

/* set(h, ids Uint32Array, status Uint8Array, inc Float64Array) -> Uint32Array of picked stash
 * indices in first-seen order — Membership.set (lib/membership/index.js:208-247) over the stash
 * the JS side kept while !isReady: mergeMembershipChangesets (merge.js:22-51) + set + checksum. */
static napi_value js_members_set(napi_env env, napi_callback_info info) {
    ARGS(4);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    size_t k = 0, k2 = 0, k3 = 0;
    const uint32_t *ids = (const uint32_t *)typed_data(env, argv[1], napi_uint32_array, &k);
    const uint8_t *st = (const uint8_t *)typed_data(env, argv[2], napi_uint8_array, &k2);
    const double *incd = (const double *)typed_data(env, argv[3], napi_float64_array, &k3);
    if ((k && (!ids || !st || !incd)) || k2 != k || k3 != k) {
        napi_throw_type_error(env, NULL, "set expects Uint32Array ids, Uint8Array status, Float64Array inc of equal length");
        return NULL;
    }
    int64_t *inc = f64_to_i64(env, incd, k, 0, "set: incarnationNumber");
    if (!inc) return NULL;
    uint32_t *pick = (uint32_t *)malloc(sizeof(uint32_t) * (k ? k : 1));
    uint32_t np = 0;
    int rc = rp_members_set((rp_members *)h->p, ids, st, inc, (uint32_t)k, pick, &np);
    free(inc);
    if (rc) {
        free(pick);
        RP_OK(rc);
    }
    void *pd = NULL;
    napi_value out = new_typed(env, napi_uint32_array, np, 4, &pd);
    if (np) memcpy(pd, pick, 4ull * np);
    free(pick);
    return out;
}

static napi_value js_members_checksum(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    uint32_t v = 0;
    int set = 0;
    RP_OK(rp_members_checksum((rp_members *)h->p, &v, &set));
    return set ? make_u32(env, v) : make_null(env);
}

static napi_value js_members_compute_checksum(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    RP_OK(rp_members_compute_checksum((rp_members *)h->p));
    return js_members_checksum(env, info);
}

static napi_value js_members_checksum_string(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    uint64_t len = 0;
    RP_OK(rp_members_checksum_string((rp_members *)h->p, NULL, 0, &len));
    char *buf = (char *)malloc(len + 1);
    int rc = rp_members_checksum_string((rp_members *)h->p, buf, len, &len);
    if (rc) {
        free(buf);
        RP_OK(rc);
    }
    napi_value s;
    napi_create_string_utf8(env, buf, len, &s);
    free(buf);
    return s;
}

/* dump(h) -> {exists: Uint8Array, status: Uint8Array, inc: Float64Array} by member id. */
static napi_value js_members_dump(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    rp_members *m = (rp_members *)h->p;
    uint32_t n = 0;
    RP_OK(rp_members_count(m, &n));
    void *ed = NULL, *sd = NULL, *id = NULL;
    napi_value ex = new_typed(env, napi_uint8_array, n, 1, &ed);
    napi_value st = new_typed(env, napi_uint8_array, n, 1, &sd);
    napi_value inc = new_typed(env, napi_float64_array, n, 8, &id);
    int64_t *i64 = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    int rc = n ? rp_members_dump(m, (uint8_t *)ed, (uint8_t *)sd, i64, n) : 0;
    for (uint32_t i = 0; rc == 0 && i < n; i++) ((double *)id)[i] = (double)i64[i];
    free(i64);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "exists", ex);
    napi_set_named_property(env, out, "status", st);
    napi_set_named_property(env, out, "inc", inc);
    return out;
}

/* ------------------------------------------------------------------ damp scoring
 * Member damp scores on the device (rp_members_damp_*; member.js:45-66,133-153,
 * membership/index.js:330-383), for the drop-in Membership (js/membership.js). */
static double prop_double(napi_env env, napi_value obj, const char *key, double dflt) {
    napi_value v;
    double d = dflt;
    if (is_nullish(env, obj) || napi_get_named_property(env, obj, key, &v) != napi_ok || is_nullish(env, v)) return dflt;
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_boolean) {
        bool b = false;
        napi_get_value_bool(env, v, &b);
        return b ? 1.0 : 0.0;
    }
    if (napi_get_value_double(env, v, &d) != napi_ok) return dflt;
    return d;
}

/* membersDampConfigure(h, {enabled, initial, min, max, penalty, suppressLimit, halfLife}) with
 * ringpop's defaults (config.js:60-71) for absent keys. */
static napi_value js_members_damp_configure(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    rp_damp_config c;
    c.enabled = prop_double(env, argv[1], "enabled", 1.0) != 0.0;
    c.initial = prop_double(env, argv[1], "initial", 0.0);
    c.min = prop_double(env, argv[1], "min", 0.0);
    c.max = prop_double(env, argv[1], "max", 10000.0);
    c.penalty = prop_double(env, argv[1], "penalty", 500.0);
    c.suppress_limit = prop_double(env, argv[1], "suppressLimit", 5000.0);
    c.half_life = prop_double(env, argv[1], "halfLife", 60.0);
    RP_OK(rp_members_damp_configure((rp_members *)h->p, &c));
    return make_null(env);
}

/* membersDampLast(h, k) -> {score: Float64Array(k), exceeded: Uint8Array(k)}: per change of the
 * last update batch, the member's dampScore after it and whether suppressLimitExceeded fired. */
static napi_value js_members_damp_last(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    uint32_t k = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &k));
    void *sd = NULL, *ed = NULL;
    napi_value sc = new_typed(env, napi_float64_array, k, 8, &sd);
    napi_value ex = new_typed(env, napi_uint8_array, k, 1, &ed);
    RP_OK(k ? rp_members_damp_last((rp_members *)h->p, (double *)sd, (uint8_t *)ed, k) : 0);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "score", sc);
    napi_set_named_property(env, out, "exceeded", ex);
    return out;
}

/* membersDampDecay(h, now): _decayMembersDampScore (index.js:374-383) on the device. */
static napi_value js_members_damp_decay(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    double now = 0;
    NAPI_OK(napi_get_value_double(env, argv[1], &now));
    int64_t *t = f64_to_i64(env, &now, 1, 0, "membersDampDecay: now");
    if (!t) return NULL;
    const int64_t now64 = t[0];
    free(t);
    RP_OK(rp_members_damp_decay((rp_members *)h->p, now64));
    return make_null(env);
}

/* membersDampDump(h) -> {score, last, ts: Float64Array (0 = null)} by member id. */
static napi_value js_members_damp_dump(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    rp_members *m = (rp_members *)h->p;
    uint32_t n = 0;
    RP_OK(rp_members_count(m, &n));
    void *sd = NULL, *ld = NULL, *td = NULL;
    napi_value sc = new_typed(env, napi_float64_array, n, 8, &sd);
    napi_value ls = new_typed(env, napi_float64_array, n, 8, &ld);
    napi_value ts = new_typed(env, napi_float64_array, n, 8, &td);
    int64_t *t64 = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    int rc = n ? rp_members_damp_dump(m, (double *)sd, (double *)ld, t64, n) : 0;
    for (uint32_t i = 0; rc == 0 && i < n; i++) ((double *)td)[i] = (double)t64[i];
    free(t64);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "score", sc);
    napi_set_named_property(env, out, "last", ls);
    napi_set_named_property(env, out, "ts", ts);
    return out;
}

/* ------------------------------------------------------------------ gossip simulator */
/* simCreate(names[], inc0 Float64Array, dead Uint8Array, seed, suspicionRounds, now0, device) */
// simCreate(names, inc0, dead, seed, suspicionRounds, now0, device[, events Uint32Array of
// (round, kind, node) triples: RP_SIM_KILL / REVIVE / LEAVE / JOIN])
static napi_value js_sim_create(napi_env env, napi_callback_info info) {
    ARGS(8);
    strpack_t s;
    if (strpack_from_array(env, argv[0], &s)) return NULL;
    size_t n1 = 0, n2 = 0;
    const double *incd = (const double *)typed_data(env, argv[1], napi_float64_array, &n1);
    const uint8_t *dead = (const uint8_t *)typed_data(env, argv[2], napi_uint8_array, &n2);
    if (!incd || !dead || n1 != s.n || n2 != s.n) {
        strpack_free(&s);
        napi_throw_type_error(env, NULL, "simCreate expects inc0 Float64Array and dead Uint8Array of names.length");
        return NULL;
    }
    uint32_t seed = 0, susp = 0;
    int32_t dev = 0;
    double now0 = 0;
    napi_get_value_uint32(env, argv[3], &seed);
    napi_get_value_uint32(env, argv[4], &susp);
    napi_get_value_double(env, argv[5], &now0);
    napi_get_value_int32(env, argv[6], &dev);
    int64_t *inc = f64_to_i64(env, incd, s.n, 0, "simCreate: inc0");
    int64_t *n0 = inc ? f64_to_i64(env, &now0, 1, 0, "simCreate: now0") : NULL;
    if (!inc || !n0) {
        free(inc);
        strpack_free(&s);
        return NULL;
    }
    const int64_t now64 = n0[0];
    free(n0);
    size_t ne = 0;
    const uint32_t *ev = NULL;
    napi_valuetype et = napi_undefined;
    if (argc > 7) napi_typeof(env, argv[7], &et);
    if (et == napi_object) {
        ev = (const uint32_t *)typed_data(env, argv[7], napi_uint32_array, &ne);
        if (!ev || ne % 3) {
            free(inc);
            strpack_free(&s);
            napi_throw_type_error(env, NULL, "simCreate events must be a Uint32Array of (round, kind, node) triples");
            return NULL;
        }
    }
    rp_sim_event *evs = (rp_sim_event *)calloc(ne / 3 + 1, sizeof(rp_sim_event));
    for (size_t i = 0; i < ne / 3; i++) {
        evs[i].round = ev[3 * i];
        evs[i].kind = ev[3 * i + 1];
        evs[i].node = ev[3 * i + 2];
    }
    rp_sim *sim = NULL;
    int rc = rp_sim_create_scenario(s.n, s.bytes, s.off32, inc, dead, seed, susp, now64, dev, NULL, 1, 0, evs,
                                    (uint32_t)(ne / 3), &sim);
    free(evs);
    free(inc);
    strpack_free(&s);
    RP_OK(rc);
    return wrap_handle(env, 3, sim);
}

static napi_value js_sim_step(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    uint32_t rounds = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &rounds));
    RP_OK(rp_sim_step((rp_sim *)h->p, rounds));
    return NULL;
}

static napi_value js_sim_round(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    int64_t r = 0;
    RP_OK(rp_sim_round((rp_sim *)h->p, &r));
    napi_value out;
    napi_create_double(env, (double)r, &out);
    return out;
}

static napi_value js_sim_checksums(napi_env env, napi_callback_info info) {
    ARGS(2);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    uint32_t n = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &n));
    void *d = NULL;
    napi_value out = new_typed(env, napi_uint32_array, n, 4, &d);
    RP_OK(rp_sim_checksums((rp_sim *)h->p, (uint32_t *)d));
    return out;
}

static napi_value js_sim_view(napi_env env, napi_callback_info info) {
    ARGS(3);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    uint32_t v = 0, n = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[1], &v));
    NAPI_OK(napi_get_value_uint32(env, argv[2], &n));
    void *sd = NULL, *id = NULL;
    napi_value st = new_typed(env, napi_uint8_array, n, 1, &sd);
    napi_value inc = new_typed(env, napi_float64_array, n, 8, &id);
    int64_t *i64 = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    int rc = rp_sim_view((rp_sim *)h->p, v, (uint8_t *)sd, i64);
    for (uint32_t i = 0; rc == 0 && i < n; i++) ((double *)id)[i] = (double)i64[i];
    free(i64);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "status", st);
    napi_set_named_property(env, out, "inc", inc);
    return out;
}

static napi_value js_sim_converged(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    int c = 0;
    RP_OK(rp_sim_converged((rp_sim *)h->p, &c));
    return make_bool(env, c);
}

static napi_value js_sim_stats(napi_env env, napi_callback_info info) {
    ARGS(1);
    handle_t *h = get_handle(env, argv[0], 3);
    if (!h) return NULL;
    uint64_t s[4] = {0, 0, 0, 0};
    RP_OK(rp_sim_stats((rp_sim *)h->p, s));
    static const char *names[4] = {"pings", "pingReqs", "fullSyncs", "applied"};
    napi_value out;
    napi_create_object(env, &out);
    for (int i = 0; i < 4; i++) {
        napi_value v;
        napi_create_double(env, (double)s[i], &v);
        napi_set_named_property(env, out, names[i], v);
    }
    return out;
}

/* ------------------------------------------------------------------ module */
/* ------------------------------------------------------------------ wire bodies */
/* the typed array at obj[key] (NULL when absent / null); *n its length */
static void *prop_typed(napi_env env, napi_value obj, const char *key, napi_typedarray_type t, size_t *n) {
    *n = 0;
    if (is_nullish(env, obj)) return NULL;
    napi_value v;
    if (napi_get_named_property(env, obj, key, &v) != napi_ok || is_nullish(env, v)) return NULL;
    return typed_data(env, v, t, n);
}

/* Incarnation numbers arrive as doubles (JS Numbers). Converting NaN, +-Inf or a value outside
 * int64 to int64_t is undefined behaviour in C, so those are rejected with a TypeError (NaN only
 * where it stands for "absent": nan_is_min). Returns NULL with the exception pending. */
static int64_t *f64_to_i64(napi_env env, const double *d, size_t n, int nan_is_min, const char *what) {
    int64_t *o = (int64_t *)malloc(sizeof(int64_t) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) {
        const double x = d[i];
        if (nan_is_min && x != x) {
            o[i] = INT64_MIN;
        } else if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) { /* NaN, Inf, range */
            char msg[160];
            snprintf(msg, sizeof msg, "%s[%zu] is not a finite number within int64 range", what, i);
            free(o);
            napi_throw_type_error(env, NULL, msg);
            return NULL;
        } else {
            o[i] = (int64_t)x;
        }
    }
    return o;
}

/* wireEncode(h, msgRecOff Uint32Array, recs {addr, src, status, inc, srcInc?, ids?}, form, body,
 * hdr {checksum?, source?, sourceInc?, target?, pingStatus?, app?}) -> {bytes: Uint8Array,
 * off: Float64Array}: JSON.stringify of the gossip bodies (dissemination.js:163-170, ping /
 * ping-req / join bodies) on the device (rp_wire_encode). inc / srcInc are Float64Array (srcInc
 * NaN = absent); src RP_NULL_ID = absent; an ids row starting with 0 = absent. */
static napi_value js_wire_encode(napi_env env, napi_callback_info info) {
    ARGS(6);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    size_t nro = 0, na = 0, ns = 0, nst = 0, ni = 0, nsi = 0, nid = 0;
    const uint32_t *ro = (const uint32_t *)typed_data(env, argv[1], napi_uint32_array, &nro);
    if (!ro || nro < 1) {
        napi_throw_type_error(env, NULL, "wireEncode expects msgRecOff Uint32Array(n_msgs + 1)");
        return NULL;
    }
    const uint32_t n_msgs = (uint32_t)(nro - 1), n_rec = ro[n_msgs];
    const uint32_t *addr = (const uint32_t *)prop_typed(env, argv[2], "addr", napi_uint32_array, &na);
    const uint32_t *src = (const uint32_t *)prop_typed(env, argv[2], "src", napi_uint32_array, &ns);
    const uint8_t *st = (const uint8_t *)prop_typed(env, argv[2], "status", napi_uint8_array, &nst);
    const double *incd = (const double *)prop_typed(env, argv[2], "inc", napi_float64_array, &ni);
    const double *sincd = (const double *)prop_typed(env, argv[2], "srcInc", napi_float64_array, &nsi);
    const uint8_t *ids = (const uint8_t *)prop_typed(env, argv[2], "ids", napi_uint8_array, &nid);
    if (na < n_rec || ns < n_rec || nst < n_rec || ni < n_rec || (sincd && nsi < n_rec) || (ids && nid < 36ull * n_rec)) {
        napi_throw_type_error(env, NULL, "wireEncode: record columns shorter than msgRecOff says");
        return NULL;
    }
    int32_t form = 0, body = 0;
    NAPI_OK(napi_get_value_int32(env, argv[3], &form));
    NAPI_OK(napi_get_value_int32(env, argv[4], &body));
    size_t hck = 0, hs = 0, hsi = 0, ht = 0, hp = 0;
    const uint32_t *ck = (const uint32_t *)prop_typed(env, argv[5], "checksum", napi_uint32_array, &hck);
    const uint32_t *ms = (const uint32_t *)prop_typed(env, argv[5], "source", napi_uint32_array, &hs);
    const double *msid = (const double *)prop_typed(env, argv[5], "sourceInc", napi_float64_array, &hsi);
    const uint32_t *tg = (const uint32_t *)prop_typed(env, argv[5], "target", napi_uint32_array, &ht);
    const uint8_t *ps = (const uint8_t *)prop_typed(env, argv[5], "pingStatus", napi_uint8_array, &hp);
    if ((ck && hck < n_msgs) || (ms && hs < n_msgs) || (msid && hsi < n_msgs) || (tg && ht < n_msgs) ||
        (ps && hp < n_msgs)) {
        napi_throw_type_error(env, NULL, "wireEncode: header columns shorter than the message count");
        return NULL;
    }
    /* the join response's app name, any length (its byte length first, then the bytes) */
    char *app = NULL;
    size_t app_len = 0;
    if (!is_nullish(env, argv[5])) {
        napi_value av;
        if (napi_get_named_property(env, argv[5], "app", &av) == napi_ok && !is_nullish(env, av)) {
            NAPI_OK(napi_get_value_string_utf8(env, av, NULL, 0, &app_len));
            app = (char *)malloc(app_len + 1);
            size_t got = 0;
            NAPI_OK(napi_get_value_string_utf8(env, av, app, app_len + 1, &got));
            app_len = got;
        }
    }
    int64_t *inc = f64_to_i64(env, incd, n_rec, 0, "wireEncode: inc");
    int64_t *sinc = (inc && sincd) ? f64_to_i64(env, sincd, n_rec, 1, "wireEncode: srcInc") : NULL;
    int64_t *msi = (inc && (!sincd || sinc) && msid) ? f64_to_i64(env, msid, n_msgs, 0, "wireEncode: sourceInc") : NULL;
    if (!inc || (sincd && !sinc) || (msid && !msi)) {
        free(inc);
        free(sinc);
        free(msi);
        free(app);
        return NULL;
    }
    rp_wire_records R = {addr, src, st, inc, sinc, ids};
    rp_wire_headers H = {ck, ms, msi, tg, ps, app_len ? app : NULL, (uint32_t)app_len};
    void *od = NULL, *bd = NULL;
    napi_value off = new_typed(env, napi_float64_array, n_msgs + 1, 8, &od);
    uint64_t *o64 = (uint64_t *)malloc(sizeof(uint64_t) * (n_msgs + 1));
    int rc = rp_wire_encode((rp_members *)h->p, n_msgs, ro, &R, form, body, &H, NULL, 0, o64);
    napi_value bytes = NULL;
    if (rc == 0) {
        bytes = new_typed(env, napi_uint8_array, o64[n_msgs] ? o64[n_msgs] : 1, 1, &bd);
        rc = rp_wire_encode((rp_members *)h->p, n_msgs, ro, &R, form, body, &H, (uint8_t *)bd, o64[n_msgs], o64);
    }
    for (uint32_t j = 0; rc == 0 && j <= n_msgs; j++) ((double *)od)[j] = (double)o64[j];
    free(inc);
    free(sinc);
    free(msi);
    free(o64);
    free(app);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    napi_set_named_property(env, out, "bytes", bytes);
    napi_set_named_property(env, out, "off", off);
    return out;
}

/* wireDecode(h, bytes Uint8Array, msgOff Float64Array(n + 1), recCap) -> {recOff, addr, src, status,
 * inc, srcInc (NaN absent), idOff, addrOff, addrLen, err, checksum, source, sourceInc (NaN absent),
 * target, pingStatus}: safeParse + the bodies' members on the device (rp_wire_decode). */
static napi_value js_wire_decode(napi_env env, napi_callback_info info) {
    ARGS(4);
    handle_t *h = get_handle(env, argv[0], 2);
    if (!h) return NULL;
    size_t nb = 0, no = 0;
    const char *buf = (const char *)typed_data(env, argv[1], napi_uint8_array, &nb);
    const double *offd = (const double *)typed_data(env, argv[2], napi_float64_array, &no);
    uint32_t cap = 0;
    NAPI_OK(napi_get_value_uint32(env, argv[3], &cap));
    if (!offd || no < 1) {
        napi_throw_type_error(env, NULL, "wireDecode expects msgOff Float64Array(n_msgs + 1)");
        return NULL;
    }
    const uint32_t n = (uint32_t)(no - 1);
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (n + 1));
    for (uint32_t j = 0; j <= n; j++) off[j] = (uint64_t)offd[j];
    if (off[n] > nb) {
        free(off);
        napi_throw_range_error(env, NULL, "wireDecode: msgOff past the buffer");
        return NULL;
    }
    const size_t c = cap ? cap : 1, m1 = n ? n : 1;
    void *p_ro, *p_a, *p_s, *p_st, *p_i, *p_si, *p_id, *p_ao, *p_al, *p_err, *p_ck, *p_ms, *p_msi, *p_tg, *p_ps;
    napi_value ro = new_typed(env, napi_uint32_array, n + 1, 4, &p_ro);
    napi_value a = new_typed(env, napi_uint32_array, c, 4, &p_a);
    napi_value s2 = new_typed(env, napi_uint32_array, c, 4, &p_s);
    napi_value st = new_typed(env, napi_uint8_array, c, 1, &p_st);
    napi_value inc = new_typed(env, napi_float64_array, c, 8, &p_i);
    napi_value sinc = new_typed(env, napi_float64_array, c, 8, &p_si);
    napi_value idoff = new_typed(env, napi_float64_array, c, 8, &p_id);
    napi_value aoff = new_typed(env, napi_float64_array, c, 8, &p_ao);
    napi_value alen = new_typed(env, napi_uint32_array, c, 4, &p_al);
    napi_value err = new_typed(env, napi_float64_array, m1, 8, &p_err);
    napi_value ck = new_typed(env, napi_uint32_array, m1, 4, &p_ck);
    napi_value ms = new_typed(env, napi_uint32_array, m1, 4, &p_ms);
    napi_value msi = new_typed(env, napi_float64_array, m1, 8, &p_msi);
    napi_value tg = new_typed(env, napi_uint32_array, m1, 4, &p_tg);
    napi_value ps = new_typed(env, napi_uint8_array, m1, 1, &p_ps);
    int64_t *i64 = (int64_t *)malloc(8 * c), *si64 = (int64_t *)malloc(8 * c), *msi64 = (int64_t *)malloc(8 * m1);
    uint64_t *id64 = (uint64_t *)malloc(8 * c), *ao64 = (uint64_t *)malloc(8 * c), *e64 = (uint64_t *)malloc(8 * m1);
    rp_wire_records_out R = {(uint32_t *)p_a, (uint32_t *)p_s, (uint8_t *)p_st, i64, si64, id64, ao64, (uint32_t *)p_al};
    rp_wire_headers_out H = {(uint32_t *)p_ck, (uint32_t *)p_ms, msi64, (uint32_t *)p_tg, (uint8_t *)p_ps};
    const int rc = rp_wire_decode((rp_members *)h->p, buf, off, n, (uint32_t *)p_ro, cap, &R, &H, e64);
    if (rc == 0) {
        const uint32_t k = ((uint32_t *)p_ro)[n] < cap ? ((uint32_t *)p_ro)[n] : cap;
        for (uint32_t r = 0; r < k; r++) {
            ((double *)p_i)[r] = (double)i64[r];
            ((double *)p_si)[r] = si64[r] == INT64_MIN ? NAN : (double)si64[r];
            ((double *)p_id)[r] = id64[r] == UINT64_MAX ? -1 : (double)id64[r];
            ((double *)p_ao)[r] = (double)ao64[r];
        }
        for (uint32_t j = 0; j < n; j++) {
            ((double *)p_err)[j] = (double)e64[j];
            ((double *)p_msi)[j] = msi64[j] == INT64_MIN ? NAN : (double)msi64[j];
        }
    }
    free(off); free(i64); free(si64); free(msi64); free(id64); free(ao64); free(e64);
    RP_OK(rc);
    napi_value out;
    napi_create_object(env, &out);
    const char *names[] = {"recOff", "addr", "src", "status", "inc", "srcInc", "idOff", "addrOff", "addrLen", "err",
                           "checksum", "source", "sourceInc", "target", "pingStatus"};
    napi_value vals[] = {ro, a, s2, st, inc, sinc, idoff, aoff, alen, err, ck, ms, msi, tg, ps};
    for (size_t i = 0; i < sizeof(vals) / sizeof(vals[0]); i++) napi_set_named_property(env, out, names[i], vals[i]);
    return out;
}

static napi_value init(napi_env env, napi_value exports) {
    static const struct {
        const char *name;
        napi_callback fn;
    } fns[] = {
        {"version", js_version},
        {"deviceCount", js_device_count},
        {"hash32", js_hash32},
        {"destroy", js_destroy},
        {"ringCreate", js_ring_create},
        {"ringAddRemove", js_ring_add_remove},
        {"ringChecksum", js_ring_checksum},
        {"ringChecksumString", js_ring_checksum_string},
        {"ringServerCount", js_ring_server_count},
        {"ringService", js_ring_service},
        {"ringLookup1", js_ring_lookup1},
        {"ringLookupN1", js_ring_lookupn1},
        {"ringTokenCount", js_ring_token_count},
        {"ringHasServer", js_ring_has_server},
        {"ringServers", js_ring_servers},
        {"ringOwnerName", js_ring_owner_name},
        {"ringLookup", js_ring_lookup},
        {"ringLookupN", js_ring_lookupn},
        {"ringLookupNHashes", js_ring_lookupn_hashes},
        {"ringGroupKeys", js_ring_group_keys},
        {"membersCreate", js_members_create},
        {"membersIntern", js_members_intern},
        {"membersSetLocal", js_members_set_local},
        {"membersUpdate", js_members_update},
        {"membersSet", js_members_set},
        {"membersChecksum", js_members_checksum},
        {"membersComputeChecksum", js_members_compute_checksum},
        {"membersChecksumString", js_members_checksum_string},
        {"membersDump", js_members_dump},
        {"membersDampConfigure", js_members_damp_configure},
        {"membersDampLast", js_members_damp_last},
        {"membersDampDecay", js_members_damp_decay},
        {"membersDampDump", js_members_damp_dump},
        {"simCreate", js_sim_create},
        {"simStep", js_sim_step},
        {"simRound", js_sim_round},
        {"simChecksums", js_sim_checksums},
        {"simView", js_sim_view},
        {"simConverged", js_sim_converged},
        {"simStats", js_sim_stats},
        {"wireEncode", js_wire_encode},
        {"wireDecode", js_wire_decode},
    };
    for (size_t i = 0; i < sizeof(fns) / sizeof(fns[0]); i++) {
        napi_value f;
        napi_create_function(env, fns[i].name, NAPI_AUTO_LENGTH, fns[i].fn, NULL, &f);
        napi_set_named_property(env, exports, fns[i].name, f);
    }
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
