// pe_graphml.cpp -- native GraphML -> edge-list ingestion.
//
// Replaces what Shadow asks igraph for before the path engine starts:
//   _topology_loadGraph          topology.c:371-399  igraph_read_graph_graphml
//   _topology_extractEdgeWeights topology.c:1212-1246 EANV("latency")
//   edge / vertex 'packetloss'   topology.c:402-444, :1442-1462 (EAN / VAN)
//   graph 'preferdirectpaths'    topology.c:769-790
// and produces exactly the ShdPeGraphDesc the engine takes: vertex ids in
// <node> document order, edge ids in <edge> document order (igraph's GraphML
// import order), endpoints as written (the engine normalises undirected
// endpoints like igraph_add_edges), numeric values correctly rounded
// (strtod), an absent or unparsable value = NaN (topology.c:330-370 treats NaN
// as "absent").  One pass over the buffer, no DOM: the only per-edge state is
// the four output arrays, so a 2*10^8-edge tmodel file is parsed at memory
// speed instead of through igraph's attribute tables.
//
// Supported XML: elements, attributes ('...' or "..."), the five predefined
// entities and numeric character references, comments, processing
// instructions, DOCTYPE, CDATA.  Namespace prefixes are ignored (GraphML's
// default namespace is the common case).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "shd_pathengine.h"

namespace {

struct Key {
    std::string forKind, name, type, deflt;
    bool hasDefault = false;
};

// a view into the input buffer
struct SV {
    const char* p = nullptr;
    size_t n = 0;
    bool eq(const char* s) const { return strlen(s) == n && memcmp(p, s, n) == 0; }
    bool eq(const SV& o) const { return o.n == n && memcmp(p, o.p, n) == 0; }
    std::string_view view() const { return std::string_view(p, n); }
};

struct Tag {
    SV name;                                            // local name
    std::vector<std::pair<SV, SV>> attrs;               // raw (entities not decoded)
    bool end = false, selfClose = false;
    const SV* raw(const char* k) const {
        for (auto& a : attrs)
            if (a.first.eq(k)) return &a.second;
        return nullptr;
    }
};

void append_utf8(std::string& o, unsigned long cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
        o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F));
        o += (char)(0x80 | (cp & 0x3F));
    } else {
        o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
        o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
    }
}

// XML entity decoding of [p, e) appended to out
void decode(const char* p, const char* e, std::string& out) {
    while (p < e) {
        const char* amp = (const char*)memchr(p, '&', (size_t)(e - p));
        if (!amp) { out.append(p, e); return; }
        out.append(p, amp);
        const char* semi = (const char*)memchr(amp, ';', (size_t)(e - amp));
        if (!semi) { out.append(amp, e); return; }
        const std::string ent(amp + 1, semi);
        if (ent == "lt") out += '<';
        else if (ent == "gt") out += '>';
        else if (ent == "amp") out += '&';
        else if (ent == "quot") out += '"';
        else if (ent == "apos") out += '\'';
        else if (!ent.empty() && ent[0] == '#') {
            const bool hex = ent.size() > 1 && (ent[1] == 'x' || ent[1] == 'X');
            append_utf8(out, strtoul(ent.c_str() + (hex ? 2 : 1), nullptr, hex ? 16 : 10));
        } else {
            out.append(amp, semi + 1);
        }
        p = semi + 1;
    }
}

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

SV local_name(const char* p, const char* e) {
    const char* colon = p;
    for (const char* q = p; q < e; ++q)
        if (*q == ':') colon = q + 1;
    return SV{colon, (size_t)(e - colon)};
}

bool has_amp(const SV& v) { return memchr(v.p, '&', v.n) != nullptr; }

// decoded attribute value ("" when absent)
std::string attr_str(const Tag& t, const char* k) {
    std::string out;
    if (const SV* v = t.raw(k)) decode(v->p, v->p + v->n, out);
    return out;
}

// Python float() on the stripped text of a view; empty / invalid -> NaN.
// strtod runs on a NUL-terminated copy (it never reads past the view) in the
// C locale Shadow runs in (a host that calls setlocale(LC_NUMERIC, ...) with
// a decimal comma would need strtod_l).
double parse_num_view(const SV& v) {
    size_t a = 0, b = v.n;
    while (a < b && is_space(v.p[a])) ++a;
    while (b > a && is_space(v.p[b - 1])) --b;
    if (a == b) return NAN;
    const char* t = v.p + a;
    const size_t len = b - a;
    const size_t k = (t[0] == '-' || t[0] == '+') ? 1 : 0;
    if (len > k + 1 && t[k] == '0' && (t[k + 1] == 'x' || t[k + 1] == 'X')) return NAN;   // no hex floats
    if (len > 64) {                         // long text: bounded copy keeps strtod inside the view
        const std::string c(t, len);
        char* end = nullptr;
        const double x = strtod(c.c_str(), &end);
        return end == c.c_str() + len ? x : NAN;
    }
    char tmp[72];
    memcpy(tmp, t, len);
    tmp[len] = 0;
    char* end = nullptr;
    const double x = strtod(tmp, &end);
    return end == tmp + len ? x : NAN;
}
double parse_num(const std::string& s) { return parse_num_view(SV{s.data(), s.size()}); }


}  // namespace

struct ShdGraphml {
    int32_t n = 0;
    int32_t directed = 1;
    int32_t prefersDirect = 0;
    bool hasVertexLoss = false;
    std::vector<int32_t> src, dst;
    std::vector<double> lat, loss, vloss;
    std::vector<std::string> ids;
};

namespace {

class Parser {
  public:
    Parser(const char* b, size_t n) : p_(b), e_(b + n) {}

    // next markup item; text before it (raw) is returned through `text`
    // returns false at end of input; sets err_ on malformed markup
    bool next(Tag& tag, const char*& t0, const char*& t1) {
        for (;;) {
            t0 = p_;
            const char* lt = (const char*)memchr(p_, '<', (size_t)(e_ - p_));
            if (!lt) { t1 = e_; p_ = e_; return false; }
            t1 = lt;
            p_ = lt + 1;
            if (p_ >= e_) { err_ = true; return false; }
            if (*p_ == '?') {                      // processing instruction
                if (!skip_past("?>")) return false;
                continue;
            }
            if (*p_ == '!') {
                if (e_ - p_ >= 3 && p_[1] == '-' && p_[2] == '-') {
                    if (!skip_past("-->")) return false;
                } else if (e_ - p_ >= 8 && memcmp(p_, "![CDATA[", 8) == 0) {
                    const char* c0 = p_ + 8;
                    if (!skip_past("]]>")) return false;
                    cdata_.append(c0, p_ - 3);
                } else {                           // DOCTYPE and friends
                    int depth = 0;
                    while (p_ < e_ && !(*p_ == '>' && depth == 0)) {
                        if (*p_ == '[') ++depth;
                        else if (*p_ == ']') --depth;
                        ++p_;
                    }
                    if (p_ >= e_) { err_ = true; return false; }
                    ++p_;
                }
                continue;
            }
            return read_tag(tag);
        }
    }
    bool error() const { return err_; }
    std::string cdata_;     // CDATA collected since the last clear

  private:
    bool skip_past(const char* s) {
        const size_t k = strlen(s);
        while (p_ + k <= e_) {
            if (memcmp(p_, s, k) == 0) { p_ += k; return true; }
            ++p_;
        }
        err_ = true;
        return false;
    }
    bool read_tag(Tag& t) {
        t.attrs.clear();
        t.end = t.selfClose = false;
        if (*p_ == '/') { t.end = true; ++p_; }
        const char* n0 = p_;
        while (p_ < e_ && !is_space(*p_) && *p_ != '>' && *p_ != '/') ++p_;
        t.name = local_name(n0, p_);
        for (;;) {
            while (p_ < e_ && is_space(*p_)) ++p_;
            if (p_ >= e_) { err_ = true; return false; }
            if (*p_ == '>') { ++p_; return true; }
            if (*p_ == '/') {
                if (p_ + 1 < e_ && p_[1] == '>') { t.selfClose = true; p_ += 2; return true; }
                err_ = true;
                return false;
            }
            const char* a0 = p_;
            while (p_ < e_ && *p_ != '=' && !is_space(*p_) && *p_ != '>') ++p_;
            const char* a1 = p_;
            while (p_ < e_ && is_space(*p_)) ++p_;
            if (p_ >= e_ || *p_ != '=') { err_ = true; return false; }
            ++p_;
            while (p_ < e_ && is_space(*p_)) ++p_;
            if (p_ >= e_ || (*p_ != '"' && *p_ != '\'')) { err_ = true; return false; }
            const char q = *p_++;
            const char* v0 = p_;
            const char* v1 = (const char*)memchr(p_, q, (size_t)(e_ - p_));
            if (!v1) { err_ = true; return false; }
            p_ = v1 + 1;
            t.attrs.emplace_back(local_name(a0, a1), SV{v0, (size_t)(v1 - v0)});
        }
    }
    const char* p_;
    const char* e_;
    bool err_ = false;
};

int parse(const char* buf, size_t len, ShdGraphml& g) {
    Parser ps(buf, len);
    Tag tag;
    const char *t0, *t1;
    std::deque<std::pair<std::string, Key>> keys;           // stable addresses
    std::unordered_map<std::string_view, int32_t> idIndex;  // views into buf or `arena`
    std::deque<std::string> arena;                           // decoded ids with entities
    std::vector<SV> stack;
    Key* curKey = nullptr;             // inside <key> (for <default>)
    const Key* dataKey = nullptr;      // key of the open <data>
    bool inGraph = false, graphDone = false, keyNodeLoss = false;
    int ctx = 0;                       // 0 none, 1 graph, 2 node, 3 edge (current owner of <data>)
    int dataDepth = -1;                // stack depth of an open <data>/<default>
    // text of the open <data>/<default>: a view while it is one entity-free
    // chunk (the common case), materialised otherwise
    int textMode = 0;                  // 0 empty, 1 view, 2 string
    SV textView;
    std::string text;
    bool inDefault = false;
    double eLat = NAN, eLoss = NAN, vLoss = NAN;
    std::string gPdp;
    bool gPdpSet = false;
    SV eSrc, eDst;
    std::string eSrcS, eDstS;          // decoded endpoints when they hold entities
    struct Pending { size_t edge; std::string src, dst; };
    std::vector<Pending> pending;
    auto find_key = [&](const SV& id) -> Key* {
        for (auto& kv : keys)
            if (kv.first.size() == id.n && memcmp(kv.first.data(), id.p, id.n) == 0) return &kv.second;
        return nullptr;
    };
    auto deflt = [&](const char* kind, const char* name, double& num, std::string* str,
                     bool* set) {
        for (auto& kv : keys) {
            const Key& k = kv.second;
            if (k.forKind == kind && k.name == name && k.hasDefault) {
                if (str) { *str = k.deflt; if (set) *set = true; }
                else num = parse_num(k.deflt);
            }
        }
    };
    auto text_add = [&](const char* p0, const char* p1) {
        if (p1 <= p0) return;
        const SV c{p0, (size_t)(p1 - p0)};
        if (textMode == 0 && !has_amp(c)) {
            textView = c;
            textMode = 1;
            return;
        }
        if (textMode == 1) text.assign(textView.p, textView.n);
        else if (textMode == 0) text.clear();
        decode(p0, p1, text);
        textMode = 2;
    };
    auto text_str = [&]() -> std::string {
        return textMode == 1 ? std::string(textView.p, textView.n)
                             : (textMode == 2 ? text : std::string());
    };
    auto text_num = [&]() -> double {
        return textMode == 1 ? parse_num_view(textView) : (textMode == 2 ? parse_num(text) : NAN);
    };
    double defLat = NAN, defLoss = NAN, defVLoss = NAN;   // fixed once <graph> opens
    auto finish_data = [&]() {
        if (!dataKey) return;
        const Key& k = *dataKey;
        if (ctx == 1 && stack.size() == 2 && k.forKind == "graph" && k.name == "preferdirectpaths") {
            gPdp = text_str();
            gPdpSet = true;
        } else if (ctx == 2) {
            if (k.name == "packetloss") vLoss = text_num();
        } else if (ctx == 3) {
            if (k.name == "latency") eLat = text_num();
            else if (k.name == "packetloss") eLoss = text_num();
        }
    };
    // an id as a lookup key: the raw view when entity-free, else decoded
    auto id_view = [&](const SV* raw, std::string& scratch) -> std::string_view {
        if (!raw) return std::string_view();
        if (!has_amp(*raw)) return raw->view();
        scratch.clear();
        decode(raw->p, raw->p + raw->n, scratch);
        return std::string_view(scratch);
    };
    for (;;) {
        const bool more = ps.next(tag, t0, t1);
        if (dataDepth >= 0) text_add(t0, t1);
        if (!ps.cdata_.empty()) {
            if (dataDepth >= 0) {
                if (textMode == 1) text.assign(textView.p, textView.n);
                else if (textMode == 0) text.clear();
                text += ps.cdata_;
                textMode = 2;
            }
            ps.cdata_.clear();
        }
        if (!more) break;
        const SV nm = tag.name;
        if (!tag.end) {
            if (nm.eq("key")) {
                Key k;
                k.forKind = attr_str(tag, "for");
                k.name = attr_str(tag, "attr.name");
                k.type = attr_str(tag, "attr.type");
                const std::string id = attr_str(tag, "id");
                if (k.forKind == "node" && k.name == "packetloss") keyNodeLoss = true;
                const SV idv{id.data(), id.size()};
                Key* ex = find_key(idv);
                if (ex) *ex = k;
                else { keys.emplace_back(id, k); ex = &keys.back().second; }
                curKey = ex;
            } else if (nm.eq("default") && curKey) {
                inDefault = true;
                dataDepth = (int)stack.size();
                textMode = 0;
            } else if (nm.eq("graph") && !graphDone && !inGraph && stack.size() == 1) {
                inGraph = true;
                ctx = 1;
                const SV* ed = tag.raw("edgedefault");
                g.directed = !ed || attr_str(tag, "edgedefault") == "directed";
                deflt("graph", "preferdirectpaths", vLoss, &gPdp, &gPdpSet);
                deflt("edge", "latency", defLat, nullptr, nullptr);
                deflt("edge", "packetloss", defLoss, nullptr, nullptr);
                deflt("node", "packetloss", defVLoss, nullptr, nullptr);
            } else if (inGraph && nm.eq("node") && stack.size() == 2) {
                ctx = 2;
                vLoss = defVLoss;
                const SV* raw = tag.raw("id");
                std::string_view key;
                if (!raw) {
                    key = std::string_view();
                } else if (!has_amp(*raw)) {
                    key = raw->view();
                } else {
                    arena.emplace_back();
                    decode(raw->p, raw->p + raw->n, arena.back());
                    key = arena.back();
                }
                if (!idIndex.emplace(key, (int32_t)g.ids.size()).second) return SHD_PE_EINVAL;
                g.ids.emplace_back(key);
            } else if (inGraph && nm.eq("edge") && stack.size() == 2) {
                ctx = 3;
                eLat = defLat;
                eLoss = defLoss;
                const SV* rs = tag.raw("source");
                const SV* rd = tag.raw("target");
                eSrc = rs ? *rs : SV{"", 0};
                eDst = rd ? *rd : SV{"", 0};
            } else if (inGraph && nm.eq("data") && ctx != 0) {
                const SV* kr = tag.raw("key");
                if (kr && has_amp(*kr)) {
                    const std::string kd = attr_str(tag, "key");
                    dataKey = find_key(SV{kd.data(), kd.size()});
                } else {
                    dataKey = kr ? find_key(*kr) : find_key(SV{"", 0});
                }
                dataDepth = (int)stack.size();
                textMode = 0;
            }
            if (tag.selfClose) {
                // an empty element: close it right away
                if (nm.eq("data") && dataDepth == (int)stack.size()) {
                    finish_data();
                    dataDepth = -1;
                } else if (nm.eq("default") && inDefault) {
                    curKey->deflt.clear();
                    curKey->hasDefault = false;    // ElementTree: text None -> no default
                    inDefault = false;
                    dataDepth = -1;
                }
                tag.end = true;                    // fall through to the close logic
            } else {
                stack.push_back(nm);
                continue;
            }
        } else {
            if (stack.empty() || !stack.back().eq(nm)) return SHD_PE_EINVAL;
            stack.pop_back();
        }
        // ---- close of element `nm` at depth stack.size() ----
        if (nm.eq("data") && dataDepth == (int)stack.size()) {
            finish_data();
            dataDepth = -1;
        } else if (nm.eq("default") && inDefault) {
            curKey->deflt = text_str();
            curKey->hasDefault = !curKey->deflt.empty();   // ElementTree: no text -> None
            inDefault = false;
            dataDepth = -1;
        } else if (nm.eq("key")) {
            curKey = nullptr;
        } else if (nm.eq("node") && ctx == 2 && stack.size() == 2) {
            g.vloss.push_back(vLoss);
            ctx = 1;
        } else if (nm.eq("edge") && ctx == 3 && stack.size() == 2) {
            // endpoints may name nodes declared later in the document
            const std::string_view sv = id_view(&eSrc, eSrcS), dv = id_view(&eDst, eDstS);
            auto a = idIndex.find(sv), b = idIndex.find(dv);
            if (a == idIndex.end() || b == idIndex.end())
                pending.push_back({g.src.size(), std::string(sv), std::string(dv)});
            g.src.push_back(a == idIndex.end() ? -1 : a->second);
            g.dst.push_back(b == idIndex.end() ? -1 : b->second);
            g.lat.push_back(eLat);
            g.loss.push_back(eLoss);
            ctx = 1;
        } else if (nm.eq("graph") && inGraph && stack.size() == 1) {
            inGraph = false;
            graphDone = true;
            ctx = 0;
        }
    }
    if (ps.error() || !stack.empty() || !graphDone) return SHD_PE_EINVAL;
    for (const auto& pe : pending) {
        auto a = idIndex.find(pe.src), b = idIndex.find(pe.dst);
        if (a == idIndex.end() || b == idIndex.end()) return SHD_PE_EINVAL;
        g.src[pe.edge] = a->second;
        g.dst[pe.edge] = b->second;
    }
    g.n = (int32_t)g.ids.size();
    g.hasVertexLoss = keyNodeLoss;
    if (gPdpSet && !gPdp.empty()) {
        std::string low;
        for (char c : gPdp) low += (char)tolower((unsigned char)c);
        g.prefersDirect = low.rfind("true", 0) == 0 || low.rfind("yes", 0) == 0 ||
                          low.rfind("1", 0) == 0;
    }
    return SHD_PE_OK;
}

}  // namespace

extern "C" int shd_graphml_parse(const char* buf, int64_t len, ShdGraphml** out) {
    if (!buf || len < 0 || !out) return SHD_PE_EINVAL;
    *out = nullptr;
    ShdGraphml* g = new (std::nothrow) ShdGraphml();
    if (!g) return SHD_PE_ENOMEM;
    int rc;
    try {
        rc = parse(buf, (size_t)len, *g);
    } catch (const std::bad_alloc&) {
        rc = SHD_PE_ENOMEM;
    }
    if (rc) { delete g; return rc; }
    *out = g;
    return SHD_PE_OK;
}

extern "C" int shd_graphml_describe(const ShdGraphml* g, ShdPeGraphDesc* desc,
                                    int32_t* prefersDirectPaths) {
    if (!g || !desc) return SHD_PE_EINVAL;
    desc->nVertices = g->n;
    desc->nEdges = (int64_t)g->src.size();
    desc->directed = g->directed;
    desc->edgeFrom = g->src.data();
    desc->edgeTo = g->dst.data();
    desc->edgeLatency = g->lat.data();
    desc->edgePacketLoss = g->loss.data();
    desc->vertexPacketLoss = g->hasVertexLoss ? g->vloss.data() : nullptr;
    if (prefersDirectPaths) *prefersDirectPaths = g->prefersDirect;
    return SHD_PE_OK;
}

extern "C" const char* shd_graphml_vertex_id(const ShdGraphml* g, int32_t v) {
    if (!g || v < 0 || v >= g->n) return nullptr;
    return g->ids[(size_t)v].c_str();
}

extern "C" void shd_graphml_free(ShdGraphml* g) { delete g; }
