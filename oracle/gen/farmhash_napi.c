/*
 * farmhash_napi.c — N-API module exposing the oracle's farmhash restatement under the
 * module name `farmhash`, so the reference JS (which does require('farmhash') at
 * lib/ring/index.js:21 and lib/membership/index.js:24) runs in THIS container to produce
 * golden vectors. TEST INFRASTRUCTURE ONLY; built into oracle/_ref/ by oracle/Makefile.
 * hash32(str) hashes the UTF-8 bytes of str and returns an unsigned 32-bit Number, the
 * contract of npm farmhash ^0.2.0 (reference package.json:34).
 */
#include <node_api.h>
#include <stdlib.h>

#include "../oracle.h"

static napi_value hash32(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    napi_get_cb_info(env, info, &argc, argv, NULL, NULL);
    size_t len = 0;
    if (argc < 1 || napi_get_value_string_utf8(env, argv[0], NULL, 0, &len) != napi_ok) {
        napi_throw_type_error(env, NULL, "hash32 expects a string");
        return NULL;
    }
    char *buf = (char *)malloc(len + 1);
    napi_get_value_string_utf8(env, argv[0], buf, len + 1, &len);
    uint32_t h = orc_hash32((const uint8_t *)buf, len);
    free(buf);
    napi_value out;
    napi_create_uint32(env, h, &out);
    return out;
}

static napi_value init(napi_env env, napi_value exports) {
    napi_value fn;
    napi_create_function(env, "hash32", NAPI_AUTO_LENGTH, hash32, NULL, &fn);
    napi_set_named_property(env, exports, "hash32", fn);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
