/* ORACLE (test infrastructure only) — minimal JSON DOM used by the CPU restatement.
 * Numbers keep their source text so that arbitrary-precision integers can be reduced
 * mod p exactly as aeson's Integer parser + mkGoldilocks do (Goldilocks.hs:98-102). */
#ifndef OR_JSON_H
#define OR_JSON_H
#include <stddef.h>

typedef enum { OJ_NULL, OJ_BOOL, OJ_NUM, OJ_STR, OJ_ARR, OJ_OBJ } oj_kind;

typedef struct oj {
  oj_kind kind;
  int boolean;
  const char* text; size_t len;   /* number text or (unescaped) string */
  struct oj** items; size_t n;    /* array elements / object values    */
  const char** keys;              /* object keys (NUL-terminated)      */
} oj;

/* parse; returns NULL on syntax error.  All memory belongs to the arena `a`. */
typedef struct oj_arena { char* buf; size_t used, cap; struct oj_arena* next; } oj_arena;
oj*  oj_parse(const char* s, size_t len, oj_arena** a);
void oj_arena_free(oj_arena* a);
oj*  oj_get(const oj* o, const char* key);   /* NULL if missing / not an object */

#endif
