/* ORACLE (test infrastructure only) — minimal recursive-descent JSON parser. */
#include "or_json.h"
#include <stdlib.h>
#include <string.h>

static void* ar_alloc(oj_arena** a, size_t sz) {
  sz = (sz + 15) & ~(size_t)15;
  if (!*a || (*a)->used + sz > (*a)->cap) {
    size_t cap = sz > (1u << 20) ? sz : (1u << 20);
    oj_arena* n = (oj_arena*)malloc(sizeof(oj_arena));
    n->buf = (char*)malloc(cap); n->used = 0; n->cap = cap; n->next = *a; *a = n;
  }
  void* p = (*a)->buf + (*a)->used; (*a)->used += sz; return p;
}

void oj_arena_free(oj_arena* a) {
  while (a) { oj_arena* n = a->next; free(a->buf); free(a); a = n; }
}

typedef struct { const char* s; size_t i, n; oj_arena** a; int err; } P;

static void ws(P* p) { while (p->i < p->n && (p->s[p->i] == ' ' || p->s[p->i] == '\n' || p->s[p->i] == '\r' || p->s[p->i] == '\t')) p->i++; }

static oj* val(P* p);

static oj* mk(P* p, oj_kind k) { oj* o = (oj*)ar_alloc(p->a, sizeof(oj)); memset(o, 0, sizeof(oj)); o->kind = k; return o; }

static char* str_raw(P* p, size_t* outlen) {
  /* p->s[p->i] == '"' */
  p->i++;
  size_t cap = 64, len = 0; char* out = (char*)malloc(cap);
  while (p->i < p->n && p->s[p->i] != '"') {
    char c = p->s[p->i++];
    if (c == '\\') {
      if (p->i >= p->n) { p->err = 1; break; }
      char e = p->s[p->i++];
      switch (e) {
        case 'n': c = '\n'; break; case 't': c = '\t'; break; case 'r': c = '\r'; break;
        case 'b': c = '\b'; break; case 'f': c = '\f'; break;
        case 'u': { /* only ASCII escapes are meaningful for our inputs */
          if (p->i + 4 > p->n) { p->err = 1; break; }
          unsigned v = (unsigned)strtoul((char[]){p->s[p->i], p->s[p->i+1], p->s[p->i+2], p->s[p->i+3], 0}, NULL, 16);
          p->i += 4; c = (char)(v < 128 ? v : '?'); break; }
        default: c = e; break;
      }
    }
    if (len + 1 >= cap) { cap *= 2; out = (char*)realloc(out, cap); }
    out[len++] = c;
  }
  if (p->i >= p->n) { p->err = 1; free(out); return NULL; }
  p->i++; /* closing quote */
  char* r = (char*)ar_alloc(p->a, len + 1); memcpy(r, out, len); r[len] = 0; free(out);
  *outlen = len; return r;
}

static oj* val(P* p) {
  ws(p);
  if (p->i >= p->n) { p->err = 1; return NULL; }
  char c = p->s[p->i];
  if (c == '{') {
    p->i++; oj* o = mk(p, OJ_OBJ);
    size_t cap = 8; oj** items = (oj**)malloc(cap * sizeof(oj*)); const char** keys = (const char**)malloc(cap * sizeof(char*));
    ws(p);
    if (p->i < p->n && p->s[p->i] == '}') { p->i++; }
    else for (;;) {
      ws(p); if (p->i >= p->n || p->s[p->i] != '"') { p->err = 1; break; }
      size_t kl; char* k = str_raw(p, &kl); if (!k) break;
      ws(p); if (p->i >= p->n || p->s[p->i] != ':') { p->err = 1; break; } p->i++;
      oj* v = val(p); if (!v) break;
      if (o->n == cap) { cap *= 2; items = (oj**)realloc(items, cap * sizeof(oj*)); keys = (const char**)realloc(keys, cap * sizeof(char*)); }
      items[o->n] = v; keys[o->n] = k; o->n++;
      ws(p); if (p->i < p->n && p->s[p->i] == ',') { p->i++; continue; }
      if (p->i < p->n && p->s[p->i] == '}') { p->i++; break; }
      p->err = 1; break;
    }
    o->items = (oj**)ar_alloc(p->a, (o->n + 1) * sizeof(oj*)); memcpy(o->items, items, o->n * sizeof(oj*));
    o->keys = (const char**)ar_alloc(p->a, (o->n + 1) * sizeof(char*)); memcpy(o->keys, keys, o->n * sizeof(char*));
    free(items); free(keys);
    return p->err ? NULL : o;
  }
  if (c == '[') {
    p->i++; oj* o = mk(p, OJ_ARR);
    size_t cap = 16; oj** items = (oj**)malloc(cap * sizeof(oj*));
    ws(p);
    if (p->i < p->n && p->s[p->i] == ']') { p->i++; }
    else for (;;) {
      oj* v = val(p); if (!v) break;
      if (o->n == cap) { cap *= 2; items = (oj**)realloc(items, cap * sizeof(oj*)); }
      items[o->n++] = v;
      ws(p); if (p->i < p->n && p->s[p->i] == ',') { p->i++; continue; }
      if (p->i < p->n && p->s[p->i] == ']') { p->i++; break; }
      p->err = 1; break;
    }
    o->items = (oj**)ar_alloc(p->a, (o->n + 1) * sizeof(oj*)); memcpy(o->items, items, o->n * sizeof(oj*));
    free(items);
    return p->err ? NULL : o;
  }
  if (c == '"') { oj* o = mk(p, OJ_STR); size_t l; o->text = str_raw(p, &l); o->len = l; return o->text ? o : NULL; }
  if (c == 't' && p->i + 4 <= p->n && !memcmp(p->s + p->i, "true", 4)) { p->i += 4; oj* o = mk(p, OJ_BOOL); o->boolean = 1; return o; }
  if (c == 'f' && p->i + 5 <= p->n && !memcmp(p->s + p->i, "false", 5)) { p->i += 5; oj* o = mk(p, OJ_BOOL); return o; }
  if (c == 'n' && p->i + 4 <= p->n && !memcmp(p->s + p->i, "null", 4)) { p->i += 4; return mk(p, OJ_NULL); }
  if (c == '-' || (c >= '0' && c <= '9')) {
    size_t st = p->i; p->i++;
    while (p->i < p->n) { char d = p->s[p->i]; if ((d >= '0' && d <= '9') || d == '.' || d == 'e' || d == 'E' || d == '+' || d == '-') p->i++; else break; }
    oj* o = mk(p, OJ_NUM); o->text = p->s + st; o->len = p->i - st; return o;
  }
  p->err = 1; return NULL;
}

oj* oj_parse(const char* s, size_t len, oj_arena** a) {
  P p = { s, 0, len, a, 0 };
  oj* v = val(&p);
  if (!v || p.err) return NULL;
  ws(&p);
  if (p.i != p.n) return NULL;
  return v;
}

oj* oj_get(const oj* o, const char* key) {
  if (!o || o->kind != OJ_OBJ) return NULL;
  for (size_t i = 0; i < o->n; i++) if (!strcmp(o->keys[i], key)) return o->items[i];
  return NULL;
}
