/* sg_topology.c — host-side topology stage of libshadowgpu: GraphML in,
 * device path tables out.
 *
 * Restates the parts of src/main/routing/topology.c that decide a packet's
 * latency and reliability (BASELINE.json north star: "a device-resident
 * latency/reliability matrix built from src/main/routing/topology.c path
 * results"):
 *   - GraphML vertices/edges and their attributes (topology.c:554-760): the
 *     vertex index is the order of <node> elements, as igraph's reader assigns
 *     it; keys are matched by attr.name;
 *   - the preferdirectpaths graph attribute (topology.c:760-790);
 *   - completeness (topology.c:450-552; an undirected self-loop counted once);
 *   - edge lookup (topology.c:402-444): reliability = 1 - packetloss;
 *   - direct paths (topology.c:1877-1927): rel = 1 * (1-lossSrcV) *
 *     (1-lossDstV) * rel(edge), latency = 0 + edge latency;
 *   - shortest paths from a source to every attached vertex
 *     (topology.c:1655-1875: igraph_get_shortest_paths_dijkstra, latency
 *     weights) and their properties (topology.c:1407-1523): rel starts at
 *     (1-lossSrcV), times (1-lossDstV) unless the path is the bare source,
 *     times each edge's reliability in path order; latency sums the edge
 *     latencies in path order; a 0 ms path becomes 1 ms (:1848-1852);
 *   - the shortest path to self (topology.c:1545-1653): the first incident
 *     edge of minimum latency, used twice (2 * lat, rel^2, no vertex loss);
 *   - which rule a lookup takes (topology.c:1969-2051): a complete graph, or
 *     preferdirectpaths with the vertices adjacent, is a direct path; anything
 *     else runs the source's shortest paths (self: the path to self);
 *   - host attachment with hints (topology.c:2094-2369).
 *
 * igraph is not available here.  Its Dijkstra is restated
 * with a binary heap and strict relaxation (the first parent that reaches a
 * vertex's final distance is kept), incident edges visited in edge order, so
 * shortest-path TIES in incomplete graphs are "parity unpinned" (DESIGN.md
 * §4).  Complete graphs — the bundled topology and every BASELINE.json config
 * — use direct paths only and are exact.
 */
#define _GNU_SOURCE
#include <ctype.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "shadowgpu.h"

extern void sg_set_error(const char* fmt, ...);

/* ------------------------------------------------------------------ graph -- */
enum { VA_ID, VA_IP, VA_CITY, VA_COUNTRY, VA_GEO, VA_TYPE, VA_N };

typedef struct {
    char* s[VA_N];  /* string attributes (NULL: absent) */
    double loss;    /* packetloss */
    int has_loss;
    uint64_t bw_down, bw_up;
} Vertex;

typedef struct {
    uint32_t a, b;  /* source, target */
    double latency, loss;
    int has_latency, has_loss;
} Edge;

struct sg_graph {
    uint32_t nv, ne, cap_v, cap_e;
    Vertex* v;
    Edge* e;
    int directed, prefers_direct, complete;
    /* incidence: for every vertex the edges it can leave by (out edges; both
     * endpoints when undirected), in edge order */
    uint32_t* inc_off;  /* [nv + 1] */
    uint32_t* inc;      /* edge ids */
};

static void graph_free(sg_graph* g) {
    if (!g) return;
    for (uint32_t i = 0; i < g->nv; ++i)
        for (int k = 0; k < VA_N; ++k) free(g->v[i].s[k]);
    free(g->v);
    free(g->e);
    free(g->inc_off);
    free(g->inc);
    free(g);
}

int sg_graph_free(sg_graph* g) {
    graph_free(g);
    return SG_OK;
}

static int grow(void** p, uint32_t* cap, uint32_t need, size_t elt) {
    if (need <= *cap) return 1;
    uint32_t c = *cap ? *cap : 64;
    while (c < need) c *= 2;
    void* q = realloc(*p, (size_t)c * elt);
    if (!q) return 0;
    memset((char*)q + (size_t)*cap * elt, 0, (size_t)(c - *cap) * elt);
    *p = q;
    *cap = c;
    return 1;
}

/* XML character data: the five predefined entities and numeric references. */
static char* xml_text(const char* s, size_t n) {
    char* r = (char*)malloc(n + 1);
    if (!r) return NULL;
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        const char* semi = s[i] == '&' ? memchr(s + i, ';', n - i) : NULL;
        if (!semi) {
            r[o++] = s[i];
            continue;
        }
        const size_t len = (size_t)(semi - (s + i));
        if (len == 3 && !strncmp(s + i, "&lt", 3)) r[o++] = '<';
        else if (len == 3 && !strncmp(s + i, "&gt", 3)) r[o++] = '>';
        else if (len == 4 && !strncmp(s + i, "&amp", 4)) r[o++] = '&';
        else if (len == 5 && !strncmp(s + i, "&quot", 5)) r[o++] = '"';
        else if (len == 5 && !strncmp(s + i, "&apos", 5)) r[o++] = '\'';
        else if (len > 2 && s[i + 1] == '#') {
            const long c = s[i + 2] == 'x' ? strtol(s + i + 3, NULL, 16) : strtol(s + i + 2, NULL, 10);
            r[o++] = (char)(c > 0 && c < 128 ? c : '?');
        } else {
            memcpy(r + o, s + i, len + 1);
            o += len + 1;
        }
        i += len;
    }
    r[o] = 0;
    return r;
}

/* Attribute `name` of the tag text [t, te), unescaped into *out. */
static int tag_attr(const char* t, const char* te, const char* name, char** out) {
    const size_t nl = strlen(name);
    for (const char* p = t; p + nl < te; ++p) {
        if (!(p == t || isspace((unsigned char)p[-1])) || strncmp(p, name, nl)) continue;
        const char* q = p + nl;
        while (q < te && isspace((unsigned char)*q)) ++q;
        if (q >= te || *q != '=') continue;
        ++q;
        while (q < te && isspace((unsigned char)*q)) ++q;
        if (q >= te || (*q != '"' && *q != '\'')) continue;
        const char quote = *q++;
        const char* e = memchr(q, quote, (size_t)(te - q));
        if (!e) return 0;
        *out = xml_text(q, (size_t)(e - q));
        return *out != NULL;
    }
    return 0;
}

typedef struct {
    char *id, *name;
    int for_edge, for_node, for_graph;
} Key;

typedef struct {
    const char* key;
    uint32_t idx;
} IdEntry;

static int id_cmp(const void* a, const void* b) {
    const int c = strcmp(((const IdEntry*)a)->key, ((const IdEntry*)b)->key);
    if (c) return c;
    const uint32_t x = ((const IdEntry*)a)->idx, y = ((const IdEntry*)b)->idx;
    return x < y ? -1 : x > y;
}

static int64_t id_find(const IdEntry* ids, uint32_t n, const char* key) {
    uint32_t lo = 0, hi = n;  /* first entry >= key */
    while (lo < hi) {
        const uint32_t mid = (lo + hi) / 2;
        if (strcmp(ids[mid].key, key) < 0) lo = mid + 1; else hi = mid;
    }
    return lo < n && !strcmp(ids[lo].key, key) ? (int64_t)ids[lo].idx : -1;
}

/* Edge id of (u, v) honouring directedness (igraph_get_eid): the lowest edge
 * id joining them, or -1. */
static int64_t find_edge(const sg_graph* g, uint32_t u, uint32_t v) {
    for (uint32_t k = g->inc_off[u]; k < g->inc_off[u + 1]; ++k) {
        const Edge* e = &g->e[g->inc[k]];
        if ((e->a == u && e->b == v) || (!g->directed && e->b == u && e->a == v)) return g->inc[k];
    }
    return -1;
}

static int build_incidence(sg_graph* g) {
    g->inc_off = (uint32_t*)calloc((size_t)g->nv + 1, sizeof(uint32_t));
    g->inc = (uint32_t*)malloc(((size_t)g->ne * 2 + 1) * sizeof(uint32_t));
    uint32_t* cur = (uint32_t*)malloc(((size_t)g->nv + 1) * sizeof(uint32_t));
    if (!g->inc_off || !g->inc || !cur) {
        free(cur);
        return 0;
    }
    for (uint32_t i = 0; i < g->ne; ++i) {
        g->inc_off[g->e[i].a + 1]++;
        if (!g->directed && g->e[i].b != g->e[i].a) g->inc_off[g->e[i].b + 1]++;
    }
    for (uint32_t v = 0; v < g->nv; ++v) g->inc_off[v + 1] += g->inc_off[v];
    memcpy(cur, g->inc_off, ((size_t)g->nv + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < g->ne; ++i) {  /* edge order within every list */
        g->inc[cur[g->e[i].a]++] = i;
        if (!g->directed && g->e[i].b != g->e[i].a) g->inc[cur[g->e[i].b]++] = i;
    }
    free(cur);
    return 1;
}

/* topology.c:450-552: every vertex needs >= V incident (out) edges, an
 * undirected self-loop counted once (igraph_incident lists it twice). */
static int is_complete(const sg_graph* g) {
    int64_t* cnt = (int64_t*)calloc(g->nv, sizeof(int64_t));
    if (!cnt) return 0;
    for (uint32_t i = 0; i < g->ne; ++i) {
        const Edge* e = &g->e[i];
        cnt[e->a]++;
        if (!g->directed) cnt[e->b]++;
    }
    int complete = 1;
    for (uint32_t v = 0; v < g->nv && complete; ++v) {
        int64_t c = cnt[v];
        if (!g->directed && find_edge(g, v, v) >= 0) c -= 1;
        if (c < (int64_t)g->nv) complete = 0;
    }
    free(cnt);
    return complete;
}

static int vertex_attr_of(const char* name) {
    static const char* names[VA_N] = {"id", "ip", "citycode", "countrycode", "geocode", "type"};
    for (int i = 1; i < VA_N; ++i)
        if (!strcasecmp(name, names[i])) return i;
    return -1;
}

int sg_graphml_load(const char* text, uint64_t len, sg_graph** out) {
    if (!text || !out) {
        sg_set_error("sg_graphml_load: NULL argument");
        return SG_ERR_INVAL;
    }
    *out = NULL;
    sg_graph* g = (sg_graph*)calloc(1, sizeof(sg_graph));
    Key* keys = NULL;
    uint32_t nkeys = 0, capk = 0, capn = 0;
    char** names = NULL;  /* [2 * ne] edge endpoint ids, resolved at the end */
    IdEntry* ids = NULL;
    char* prefer = NULL;
    int rc = SG_ERR_INVAL;
    if (!g) return SG_ERR_NOMEM;
    const char* p = text;
    const char* end = text + len;
    int in_graph = 0, saw_graph = 0, kind = 0;  /* kind: 1 inside <node>, 2 inside <edge> */
    uint32_t cur = 0;
    while (p < end) {
        const char* lt = memchr(p, '<', (size_t)(end - p));
        if (!lt) break;
        if (end - lt >= 4 && !strncmp(lt, "<!--", 4)) {
            const char* ce = NULL;
            for (const char* q = lt + 4; end - q >= 3; ++q)
                if (!strncmp(q, "-->", 3)) {
                    ce = q;
                    break;
                }
            if (!ce) break;
            p = ce + 3;
            continue;
        }
        if (end - lt >= 9 && !strncmp(lt, "<![CDATA[", 9)) {  /* GraphML embedded in a config */
            p = lt + 9;
            continue;
        }
        const char* gt = memchr(lt, '>', (size_t)(end - lt));
        if (!gt) {
            sg_set_error("sg_graphml_load: unterminated tag");
            goto fail;
        }
        const char* t = lt + 1;
        const int closing = *t == '/';
        const int selfclose = gt > t && gt[-1] == '/';
        if (closing) ++t;
        const char* ne = t;
        while (ne < gt && !isspace((unsigned char)*ne) && *ne != '/') ++ne;
        const size_t nlen = (size_t)(ne - t);
        p = gt + 1;
#define TAG(x) (nlen == sizeof(x) - 1 && !strncmp(t, x, nlen))
        if (*t == '?' || *t == '!') continue;
        if (TAG("key") && !closing) {
            if (!grow((void**)&keys, &capk, nkeys + 1, sizeof(Key))) goto nomem;
            Key* k = &keys[nkeys++];
            char* f = NULL;
            tag_attr(ne, gt, "id", &k->id);
            tag_attr(ne, gt, "attr.name", &k->name);
            if (tag_attr(ne, gt, "for", &f)) {
                k->for_edge = !strcmp(f, "edge");
                k->for_node = !strcmp(f, "node");
                k->for_graph = !strcmp(f, "graph");
                free(f);
            }
            if (!k->id || !k->name) {
                sg_set_error("sg_graphml_load: <key> without id or attr.name");
                goto fail;
            }
        } else if (TAG("graph")) {
            if (closing) {
                in_graph = 0;
            } else {
                if (saw_graph) {
                    sg_set_error("sg_graphml_load: more than one <graph>");
                    goto fail;
                }
                saw_graph = in_graph = 1;
                char* ed = NULL;
                if (tag_attr(ne, gt, "edgedefault", &ed)) {
                    g->directed = !strcmp(ed, "directed");
                    free(ed);
                }
            }
        } else if (TAG("node") && in_graph) {
            if (closing) {
                kind = 0;
                continue;
            }
            if (!grow((void**)&g->v, &g->cap_v, g->nv + 1, sizeof(Vertex))) goto nomem;
            if (!tag_attr(ne, gt, "id", &g->v[g->nv].s[VA_ID])) {
                sg_set_error("sg_graphml_load: <node> without id");
                goto fail;
            }
            cur = g->nv++;
            kind = selfclose ? 0 : 1;
        } else if (TAG("edge") && in_graph) {
            if (closing) {
                kind = 0;
                continue;
            }
            if (!grow((void**)&g->e, &g->cap_e, g->ne + 1, sizeof(Edge))) goto nomem;
            if (!grow((void**)&names, &capn, 2 * (g->ne + 1), sizeof(char*))) goto nomem;
            if (!tag_attr(ne, gt, "source", &names[2 * g->ne]) || !tag_attr(ne, gt, "target", &names[2 * g->ne + 1])) {
                sg_set_error("sg_graphml_load: <edge> without source or target");
                ++g->ne;  /* its names are freed below */
                goto fail;
            }
            cur = g->ne++;
            kind = selfclose ? 0 : 2;
        } else if (TAG("data") && !closing && !selfclose) {
            char* kid = NULL;
            tag_attr(ne, gt, "key", &kid);
            const char* ve = NULL;
            for (const char* q = p; end - q >= 7; ++q)
                if (!strncmp(q, "</data>", 7)) {
                    ve = q;
                    break;
                }
            if (!ve || !kid) {
                free(kid);
                sg_set_error("sg_graphml_load: malformed <data>");
                goto fail;
            }
            const Key* k = NULL;
            for (uint32_t i = 0; i < nkeys; ++i)
                if (!strcmp(keys[i].id, kid)) k = &keys[i];
            free(kid);
            char* val = k ? xml_text(p, (size_t)(ve - p)) : NULL;
            p = ve + 7;
            if (!k) continue;
            if (!val) goto nomem;
            if (kind == 1 && k->for_node) {
                Vertex* v = &g->v[cur];
                const int a = vertex_attr_of(k->name);
                if (!strcasecmp(k->name, "packetloss")) {
                    v->loss = strtod(val, NULL);
                    v->has_loss = 1;
                } else if (!strcasecmp(k->name, "bandwidthdown")) {
                    v->bw_down = strtoull(val, NULL, 10);
                } else if (!strcasecmp(k->name, "bandwidthup")) {
                    v->bw_up = strtoull(val, NULL, 10);
                } else if (a > 0) {
                    free(v->s[a]);
                    v->s[a] = val;
                    val = NULL;
                }
            } else if (kind == 2 && k->for_edge) {
                Edge* e = &g->e[cur];
                if (!strcasecmp(k->name, "latency")) {
                    e->latency = strtod(val, NULL);
                    e->has_latency = 1;
                } else if (!strcasecmp(k->name, "packetloss")) {
                    e->loss = strtod(val, NULL);
                    e->has_loss = 1;
                }
            } else if (kind == 0 && in_graph && k->for_graph && !strncasecmp(k->name, "preferdirectpaths", 17)) {
                free(prefer);
                prefer = val;
                val = NULL;
            }
            free(val);
        }
#undef TAG
    }
    if (!saw_graph || g->nv == 0) {
        sg_set_error("sg_graphml_load: no <graph> with nodes");
        goto fail;
    }
    ids = (IdEntry*)malloc((size_t)g->nv * sizeof(IdEntry));
    if (!ids) goto nomem;
    for (uint32_t i = 0; i < g->nv; ++i) {
        ids[i].key = g->v[i].s[VA_ID];
        ids[i].idx = i;
    }
    qsort(ids, g->nv, sizeof(IdEntry), id_cmp);  /* a duplicated id resolves to its first node */
    for (uint32_t i = 0; i < g->ne; ++i) {
        const int64_t a = id_find(ids, g->nv, names[2 * i]);
        const int64_t b = id_find(ids, g->nv, names[2 * i + 1]);
        if (a < 0 || b < 0) {
            sg_set_error("sg_graphml_load: edge %u names an unknown node", i);
            goto fail;
        }
        if (!g->e[i].has_latency || !g->e[i].has_loss) {  /* required edge attributes (topology.c:1588-1596) */
            sg_set_error("sg_graphml_load: edge %u lacks latency or packetloss", i);
            goto fail;
        }
        g->e[i].a = (uint32_t)a;
        g->e[i].b = (uint32_t)b;
    }
    if (prefer) {  /* topology.c:769-779 */
        g->prefers_direct = !strncasecmp(prefer, "true", 4) || !strncasecmp(prefer, "yes", 3) ||
                            !strncasecmp(prefer, "1", 1);
    }
    if (!build_incidence(g)) goto nomem;
    g->complete = is_complete(g);
    rc = SG_OK;
    goto done;
nomem:
    rc = SG_ERR_NOMEM;
    sg_set_error("sg_graphml_load: out of memory");
fail:
    graph_free(g);
    g = NULL;
done:
    for (uint32_t i = 0; i < nkeys; ++i) {
        free(keys[i].id);
        free(keys[i].name);
    }
    free(keys);
    for (uint32_t i = 0; i < capn; ++i) free(names[i]);  /* unused slots are NULL */
    free(names);
    free(ids);
    free(prefer);
    *out = g;
    return rc;
}

int sg_graph_info(const sg_graph* g, sg_graph_desc* out) {
    if (!g || !out) {
        sg_set_error("sg_graph_info: NULL argument");
        return SG_ERR_INVAL;
    }
    memset(out, 0, sizeof *out);
    out->n_vertices = g->nv;
    out->n_edges = g->ne;
    out->directed = g->directed;
    out->complete = g->complete;
    out->prefers_direct = g->prefers_direct;
    double mn = INFINITY, mx = -INFINITY;
    for (uint32_t i = 0; i < g->ne; ++i) {
        mn = g->e[i].latency < mn ? g->e[i].latency : mn;
        mx = g->e[i].latency > mx ? g->e[i].latency : mx;
    }
    out->min_edge_latency_ms = g->ne ? mn : 0;
    out->max_edge_latency_ms = g->ne ? mx : 0;
    return SG_OK;
}

int sg_graph_vertex(const sg_graph* g, uint32_t index, sg_vertex_desc* out) {
    if (!g || !out || index >= g->nv) {
        sg_set_error("sg_graph_vertex: bad argument");
        return SG_ERR_INVAL;
    }
    const Vertex* v = &g->v[index];
    out->id = v->s[VA_ID];
    out->ip = v->s[VA_IP];
    out->citycode = v->s[VA_CITY];
    out->countrycode = v->s[VA_COUNTRY];
    out->geocode = v->s[VA_GEO];
    out->type = v->s[VA_TYPE];
    out->packetloss = v->has_loss ? v->loss : 0.0;
    out->has_packetloss = v->has_loss;
    out->bandwidth_down = v->bw_down;
    out->bandwidth_up = v->bw_up;
    return SG_OK;
}

int sg_graph_edge(const sg_graph* g, uint32_t index, uint32_t* src, uint32_t* dst, double* latency_ms,
                  double* packetloss) {
    if (!g || index >= g->ne) {
        sg_set_error("sg_graph_edge: bad argument");
        return SG_ERR_INVAL;
    }
    if (src) *src = g->e[index].a;
    if (dst) *dst = g->e[index].b;
    if (latency_ms) *latency_ms = g->e[index].latency;
    if (packetloss) *packetloss = g->e[index].loss;
    return SG_OK;
}

/* ------------------------------------------------------------------ paths -- */
/* topology.c:1877-1927 */
static void direct_path(const sg_graph* g, uint32_t s, uint32_t d, int64_t eid, double* lat, double* rel) {
    double r = 1.0, l = 0.0;
    if (g->v[s].has_loss) r *= (1.0f - g->v[s].loss);
    if (g->v[d].has_loss) r *= (1.0f - g->v[d].loss);
    l += g->e[eid].latency;
    r *= (1.0f - g->e[eid].loss);
    *lat = l;
    *rel = r;
}

/* topology.c:1545-1653: the first incident edge of minimum latency, twice.
 * Returns 0 when the vertex has no incident edge. */
static int self_path(const sg_graph* g, uint32_t v, double* lat, double* rel) {
    double minLatency = 0.0f, relMin = 0.0f;
    int found = 0;
    for (uint32_t k = g->inc_off[v]; k < g->inc_off[v + 1]; ++k) {
        const Edge* e = &g->e[g->inc[k]];
        if (minLatency == 0 || e->latency < minLatency) {
            minLatency = e->latency;
            relMin = 1.0f - e->loss;
        }
        found = 1;
    }
    *lat = 2.0f * minLatency;
    *rel = relMin * relMin;
    return found;
}

typedef struct {
    double d;
    uint32_t v;
} HeapItem;

static void heap_push(HeapItem* h, uint32_t* n, HeapItem x) {
    uint32_t i = (*n)++;
    while (i > 0) {
        const uint32_t pi = (i - 1) / 2;
        if (h[pi].d < x.d || (h[pi].d == x.d && h[pi].v <= x.v)) break;
        h[i] = h[pi];
        i = pi;
    }
    h[i] = x;
}

static HeapItem heap_pop(HeapItem* h, uint32_t* n) {
    const HeapItem top = h[0];
    const HeapItem x = h[--(*n)];
    uint32_t i = 0;
    for (;;) {
        uint32_t c = 2 * i + 1;
        if (c >= *n) break;
        if (c + 1 < *n && (h[c + 1].d < h[c].d || (h[c + 1].d == h[c].d && h[c + 1].v < h[c].v))) ++c;
        if (x.d < h[c].d || (x.d == h[c].d && x.v <= h[c].v)) break;
        h[i] = h[c];
        i = c;
    }
    if (*n) h[i] = x;
    return top;
}

/* Single-source shortest paths by latency (igraph_get_shortest_paths_dijkstra
 * restated): dist[] and the parent edge of every reached vertex. */
static int dijkstra(const sg_graph* g, uint32_t s, double* dist, int64_t* parent, HeapItem* heap, uint8_t* done) {
    for (uint32_t v = 0; v < g->nv; ++v) {
        dist[v] = INFINITY;
        parent[v] = -1;
        done[v] = 0;
    }
    uint32_t n = 0;
    dist[s] = 0.0;
    heap_push(heap, &n, (HeapItem){0.0, s});
    while (n) {
        const HeapItem it = heap_pop(heap, &n);
        if (done[it.v] || it.d > dist[it.v]) continue;
        done[it.v] = 1;
        const uint32_t u = it.v;
        for (uint32_t k = g->inc_off[u]; k < g->inc_off[u + 1]; ++k) {
            const uint32_t eid = g->inc[k];
            const Edge* e = &g->e[eid];
            const uint32_t w = e->a == u ? e->b : e->a;
            if (done[w]) continue;
            const double alt = dist[u] + e->latency;
            if (alt < dist[w]) {
                dist[w] = alt;
                parent[w] = eid;
                heap_push(heap, &n, (HeapItem){alt, w});
            }
        }
    }
    return 1;
}

/* topology.c:1407-1523 for the Dijkstra path s -> t (t != s). */
static void path_props(const sg_graph* g, uint32_t s, uint32_t t, const int64_t* parent, uint32_t* stack,
                       double* lat, double* rel) {
    uint32_t n = 0;
    for (uint32_t v = t; v != s;) {  /* edges from t back to s */
        const int64_t eid = parent[v];
        stack[n++] = (uint32_t)eid;
        v = g->e[eid].a == v ? g->e[eid].b : g->e[eid].a;
    }
    double r = 1.0, l = 0.0;
    if (g->v[s].has_loss) r *= (1.0f - g->v[s].loss);
    /* nVertices = n + 1 >= 2 and s != t: the destination's loss is included */
    if (g->v[t].has_loss) r *= (1.0f - g->v[t].loss);
    while (n) {  /* path order: source first */
        const Edge* e = &g->e[stack[--n]];
        l += e->latency;
        r *= (1.0f - e->loss);
    }
    *lat = l;
    *rel = r;
}

int sg_graph_paths(const sg_graph* g, const uint8_t* attached, double* latency_ms, double* reliability,
                   double* discovered_ms, uint8_t* kind) {
    if (!g || !latency_ms || !reliability) {
        sg_set_error("sg_graph_paths: NULL argument");
        return SG_ERR_INVAL;
    }
    const uint32_t V = g->nv;
    double* dist = (double*)malloc((size_t)V * sizeof(double));
    int64_t* parent = (int64_t*)malloc((size_t)V * sizeof(int64_t));
    HeapItem* heap = (HeapItem*)malloc(((size_t)g->ne * 2 + V + 1) * sizeof(HeapItem));
    uint8_t* done = (uint8_t*)malloc(V);
    uint32_t* stack = (uint32_t*)malloc(((size_t)V + 1) * sizeof(uint32_t));
    if (!dist || !parent || !heap || !done || !stack) {
        free(dist);
        free(parent);
        free(heap);
        free(done);
        free(stack);
        sg_set_error("sg_graph_paths: out of memory");
        return SG_ERR_NOMEM;
    }
    int rc = SG_OK;
    for (uint32_t s = 0; s < V && rc == SG_OK; ++s) {
        int ran = 0;  /* this source's shortest paths computed */
        double srcmin = INFINITY;  /* min latency over the paths a source run stores */
        for (uint32_t d = 0; d < V; ++d) {
            const size_t k = (size_t)s * V + d;
            const int64_t eid = find_edge(g, s, d);
            double l = NAN, r = NAN;
            uint8_t how;
            if (g->complete || (g->prefers_direct && eid >= 0)) {
                if (eid < 0) {
                    sg_set_error("sg_graph_paths: no edge %u -> %u in a complete graph", s, d);
                    rc = SG_ERR_INVAL;
                    break;
                }
                direct_path(g, s, d, eid, &l, &r);
                how = SG_PATH_DIRECT;
            } else if (s == d) {
                if (!self_path(g, s, &l, &r)) {
                    sg_set_error("sg_graph_paths: vertex %u has no incident edge", s);
                    rc = SG_ERR_INVAL;
                    break;
                }
                how = SG_PATH_SELF;
            } else {
                if (!ran) {
                    dijkstra(g, s, dist, parent, heap, done);
                    ran = 1;
                    /* every attached target's path is stored at once (topology.c:1805-1864),
                     * except where a direct path is preferred (topology.c:1325-1331) */
                    for (uint32_t t = 0; t < V; ++t) {
                        if (t == s || (attached && !attached[t]) || !isfinite(dist[t])) continue;
                        if (g->prefers_direct && find_edge(g, s, t) >= 0) continue;
                        double lt, rt;
                        path_props(g, s, t, parent, stack, &lt, &rt);
                        if (lt == 0) lt = 1;
                        srcmin = lt < srcmin ? lt : srcmin;
                    }
                }
                if (!isfinite(dist[d])) {
                    sg_set_error("sg_graph_paths: vertex %u unreachable from %u", d, s);
                    rc = SG_ERR_INVAL;
                    break;
                }
                path_props(g, s, d, parent, stack, &l, &r);
                if (l == 0) l = 1;  /* topology.c:1848-1852 */
                how = SG_PATH_SHORTEST;
            }
            latency_ms[k] = l;
            reliability[k] = r;
            if (kind) kind[k] = how;
            if (discovered_ms) discovered_ms[k] = how == SG_PATH_SHORTEST ? srcmin : l;
        }
    }
    free(dist);
    free(parent);
    free(heap);
    free(done);
    free(stack);
    return rc;
}

/* ----------------------------------------------------------------- attach -- */
/* inet_addr-style dotted quad in network byte order (address_stringToIP);
 * INADDR_NONE (0xFFFFFFFF) when it does not parse. */
static uint32_t ip_of(const char* s) {
    unsigned b[4];
    char tail;
    if (!s || sscanf(s, "%u.%u.%u.%u%c", &b[0], &b[1], &b[2], &b[3], &tail) != 4) return 0xFFFFFFFFu;
    for (int i = 0; i < 4; ++i)
        if (b[i] > 255) return 0xFFFFFFFFu;
    return (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

static int usable_ip(uint32_t ip) {  /* not INADDR_NONE, INADDR_ANY, INADDR_LOOPBACK */
    return ip != 0xFFFFFFFFu && ip != 0 && ip != 0x0100007Fu;
}

static int eq_hint(const char* attr, const char* hint) { return attr && hint && !strcasecmp(attr, hint); }

int sg_graph_attach(const sg_graph* g, uint32_t n_hosts, const sg_attach_hint* hints, uint32_t* rng_state,
                    uint32_t* vertex_out) {
    if (!g || !rng_state || !vertex_out) {
        sg_set_error("sg_graph_attach: NULL argument");
        return SG_ERR_INVAL;
    }
    const uint32_t V = g->nv;
    /* candidate queues: city+type, city, country+type, country, geo+type, geo, type, all */
    enum { Q_CT, Q_C, Q_NT, Q_N, Q_GT, Q_G, Q_T, Q_ALL, NQ };
    uint32_t* q = (uint32_t*)malloc((size_t)NQ * V * sizeof(uint32_t));
    if (!q) {
        sg_set_error("sg_graph_attach: out of memory");
        return SG_ERR_NOMEM;
    }
    for (uint32_t h = 0; h < n_hosts; ++h) {
        const sg_attach_hint* a = hints ? &hints[h] : NULL;
        const char* iph = a ? a->ip : NULL;
        const uint32_t req = iph ? ip_of(iph) : 0xFFFFFFFFu;
        const int req_usable = iph && usable_ip(req);
        uint32_t nq[NQ] = {0}, nip[NQ] = {0};
        int exact = 0;
        for (uint32_t v = 0; v < V; ++v) {  /* topology.c:2094-2217 */
            const Vertex* x = &g->v[v];
            const int city = eq_hint(x->s[VA_CITY], a ? a->citycode : NULL);
            const int country = eq_hint(x->s[VA_COUNTRY], a ? a->countrycode : NULL);
            const int geo = eq_hint(x->s[VA_GEO], a ? a->geocode : NULL);
            const int type = eq_hint(x->s[VA_TYPE], a ? a->type : NULL);
            const uint32_t vip = x->s[VA_IP] ? ip_of(x->s[VA_IP]) : 0xFFFFFFFFu;
            const int vusable = x->s[VA_IP] && usable_ip(vip);
            if (req_usable && vusable && vip == req) {
                if (!exact) memset(nq, 0, sizeof nq), memset(nip, 0, sizeof nip);
                exact = 1;
                q[Q_ALL * V + nq[Q_ALL]++] = v;
                nip[Q_ALL] += vusable;
            }
            if (exact) continue;
            q[Q_ALL * V + nq[Q_ALL]++] = v;
            nip[Q_ALL] += vusable;
            const int m[NQ] = {city && type, city, country && type, country, geo && type, geo, type, 0};
            for (int i = 0; i < Q_ALL; ++i)
                if (m[i]) {
                    q[i * V + nq[i]++] = v;
                    nip[i] += vusable;
                }
        }
        int sel = Q_ALL;  /* topology.c:2290-2317 */
        for (int i = 0; i < Q_ALL; ++i)
            if (nq[i] > 0) {
                sel = i;
                break;
            }
        const int lpm = sel == Q_ALL ? (iph && nip[Q_ALL] > 0) : (req_usable && nip[sel] > 0);
        const uint32_t* cand = q + (size_t)sel * V;
        uint32_t chosen;
        if (lpm && !exact) {  /* topology.c:2219-2246 */
            uint32_t best = 0;
            chosen = cand[0];
            for (uint32_t i = 0; i < nq[sel]; ++i) {
                const uint32_t vip = ip_of(g->v[cand[i]].s[VA_IP]);
                const uint32_t match = ~(vip ^ req);
                if (match > best || best == 0) {
                    best = match;
                    chosen = cand[i];
                }
            }
        } else {  /* topology.c:2327-2333 */
            const double r = sg_random_next_double(&rng_state[h]);
            const int range = (int)nq[sel] - 1;
            const int idx = (int)round((double)(range * r));
            chosen = cand[idx];
        }
        vertex_out[h] = chosen;
    }
    free(q);
    return SG_OK;
}

/* Device tables from path latencies / reliabilities (worker.c:268-277,
 * master.c:153): delay = ceil(latency * 1e6), keep threshold, truncated ms. */
int sg_build_path_tables(uint32_t n_vertices, const double* latency_ms, const double* reliability,
                         const double* discovered_ms, uint64_t* delay_ns, int32_t* keep_max, uint32_t* jump_ms) {
    if (!latency_ms || !reliability || !delay_ns || !keep_max || !jump_ms || n_vertices == 0) {
        sg_set_error("sg_build_path_tables: bad argument");
        return SG_ERR_INVAL;
    }
    const size_t n = (size_t)n_vertices * n_vertices;
    for (size_t i = 0; i < n; ++i) {
        const double l = latency_ms[i];
        if (!(l >= 0) || !(l < 1e9)) {
            sg_set_error("sg_build_path_tables: latency %g ms out of range at %zu", l, i);
            return SG_ERR_INVAL;
        }
        delay_ns[i] = (uint64_t)ceil(l * 1000000.0);
        keep_max[i] = sg_keep_threshold(reliability[i]);
        const double j = discovered_ms ? discovered_ms[i] : l;
        jump_ms[i] = (uint32_t)(uint64_t)j;
    }
    return SG_OK;
}

/* ------------------------------------------------------------ path cache -- */
struct sg_path_cache {
    uint32_t V;
    int complete, directed;
    double* lat;        /* [V*V] the latency a store caches */
    uint8_t* kind;      /* [V*V] sg_path_kind */
    uint8_t* cached;    /* [V*V] entry stored for (src, dst) */
    uint32_t* targets;  /* attached vertices (_topology_getUniqueVertexTargets) */
    uint32_t nt;
    double min_ms;      /* topology->minimumPathLatency, 0 = unset */
    uint64_t runs, stored;
};

int sg_path_cache_create(uint32_t V, const double* latency_ms, const uint8_t* kind, const uint8_t* attached,
                         int complete, int directed, sg_path_cache** out) {
    if (!out || !latency_ms || !kind || V == 0) {
        sg_set_error("sg_path_cache_create: bad argument");
        return SG_ERR_INVAL;
    }
    *out = NULL;
    const size_t n = (size_t)V * V;
    sg_path_cache* c = (sg_path_cache*)calloc(1, sizeof *c);
    if (c) {
        c->lat = (double*)malloc(n * sizeof(double));
        c->kind = (uint8_t*)malloc(n);
        c->cached = (uint8_t*)calloc(n, 1);
        c->targets = (uint32_t*)malloc((size_t)V * 4);
    }
    if (!c || !c->lat || !c->kind || !c->cached || !c->targets) {
        sg_path_cache_destroy(c);
        sg_set_error("sg_path_cache_create: out of memory");
        return SG_ERR_NOMEM;
    }
    c->V = V;
    c->complete = complete;
    c->directed = directed;
    memcpy(c->lat, latency_ms, n * sizeof(double));
    memcpy(c->kind, kind, n);
    for (uint32_t v = 0; v < V; ++v)
        if (!attached || attached[v]) c->targets[c->nt++] = v;
    *out = c;
    return SG_OK;
}

int sg_path_cache_destroy(sg_path_cache* c) {
    if (!c) return SG_OK;
    free(c->lat);
    free(c->kind);
    free(c->cached);
    free(c->targets);
    free(c);
    return SG_OK;
}

/* _topology_storePathInCache (topology.c:1337-1390) behind
 * _topology_shouldStorePath (1306-1336). */
static void pc_store(sg_path_cache* c, int direct, uint32_t s, uint32_t t) {
    const size_t k = (size_t)s * c->V + t, kr = (size_t)t * c->V + s;
    if (c->cached[k] || c->cached[kr]) return;               /* either direction: 1312-1318 */
    if (c->complete && !direct) return;                      /* 1321-1323 */
    if (!direct && c->kind[k] == SG_PATH_DIRECT) return;     /* preferred direct edge: 1325-1331 */
    c->cached[k] = 1;
    c->stored++;
    const double l = c->lat[k];
    if (c->min_ms == 0 || l < c->min_ms) c->min_ms = l;      /* 1374-1385 */
}

int sg_path_cache_lookup(sg_path_cache* c, uint32_t s, uint32_t d, uint64_t* pair_out, double* min_ms_out) {
    if (!c || !pair_out || s >= c->V || d >= c->V) {
        sg_set_error("sg_path_cache_lookup: bad argument");
        return SG_ERR_INVAL;
    }
    const uint32_t V = c->V;
    const size_t k = (size_t)s * V + d, kr = (size_t)d * V + s;
    if (!c->cached[k] && (c->directed || !c->cached[kr])) {  /* a miss: topology.c:1986-1990 */
        if (c->kind[k] == SG_PATH_DIRECT) {
            pc_store(c, 1, s, d);                            /* 2013-2024 */
        } else if (s == d) {
            pc_store(c, 0, s, s);                            /* the self path, stored as non-direct (1650) */
        } else {                                             /* one Dijkstra run from s: 1655-1875 */
            c->runs++;
            for (uint32_t i = 0; i < c->nt; ++i)
                if (c->targets[i] != s) pc_store(c, 0, s, c->targets[i]);
        }
        if (!c->cached[k] && !c->cached[kr]) {               /* 2033-2045 */
            sg_set_error("sg_path_cache_lookup: no path %u -> %u after the lookup", s, d);
            return SG_ERR_STATE;
        }
    }
    *pair_out = c->cached[k] ? k : kr;                       /* 2033-2036: either direction after a miss */
    if (min_ms_out) *min_ms_out = c->min_ms;
    return SG_OK;
}

int sg_path_cache_stats(const sg_path_cache* c, uint64_t* runs, uint64_t* stored) {
    if (!c) return SG_ERR_INVAL;
    if (runs) *runs = c->runs;
    if (stored) *stored = c->stored;
    return SG_OK;
}
