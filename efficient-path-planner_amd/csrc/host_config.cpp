// host_config.cpp — ConfigParser (src/ConfigParserYAML.cpp:10-118) over small
// order-preserving JSON and block-YAML readers.  Object members keep document order,
// which is the iteration order yaml-cpp gives the reference for component_geometry.
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "epp/ConfigParser.h"

namespace epp {

class JsonValue {
public:
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<JsonValue> arr;
    std::vector<std::pair<std::string, JsonValue>> obj;

    const JsonValue* find(const std::string& k) const {
        for (const auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

namespace {

class Reader {
public:
    explicit Reader(const std::string& s) : s_(s) {}
    JsonValue parse() {
        JsonValue v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    [[noreturn]] void fail(const std::string& m) {
        throw std::runtime_error("config JSON parse error at offset " + std::to_string(i_) + ": " + m);
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\t' || s_[i_] == '\r')) ++i_;
    }
    bool lit(const char* t) {
        size_t n = std::char_traits<char>::length(t);
        if (s_.compare(i_, n, t) == 0) {
            i_ += n;
            return true;
        }
        return false;
    }
    std::string string() {
        if (s_[i_] != '"') fail("expected string");
        ++i_;
        std::string out;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) fail("bad escape");
                char e = s_[i_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': i_ += 4; out += '?'; break;
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return out;
    }
    JsonValue value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        JsonValue v;
        char c = s_[i_];
        if (c == '{') {
            v.kind = JsonValue::Object;
            ++i_;
            ws();
            if (s_[i_] == '}') {
                ++i_;
                return v;
            }
            while (true) {
                ws();
                std::string k = string();
                ws();
                if (s_[i_] != ':') fail("expected ':'");
                ++i_;
                v.obj.emplace_back(k, value());
                ws();
                if (s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (s_[i_] == '}') {
                    ++i_;
                    break;
                }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            v.kind = JsonValue::Array;
            ++i_;
            ws();
            if (s_[i_] == ']') {
                ++i_;
                return v;
            }
            while (true) {
                v.arr.push_back(value());
                ws();
                if (s_[i_] == ',') {
                    ++i_;
                    continue;
                }
                if (s_[i_] == ']') {
                    ++i_;
                    break;
                }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.kind = JsonValue::String;
            v.str = string();
        } else if (lit("true")) {
            v.kind = JsonValue::Bool;
            v.b = true;
            v.str = "true";  // (yaml-cpp reads a JSON scalar's text as the string)
        } else if (lit("false")) {
            v.kind = JsonValue::Bool;
            v.b = false;
            v.str = "false";
        } else if (lit("null")) {
            v.kind = JsonValue::Null;
        } else {
            char* end = nullptr;
            const char* at = s_.c_str() + i_;
            v.num = std::strtod(at, &end);
            if (end == at) fail("bad value");
            v.str.assign(at, (size_t)(end - at));
            i_ = end - s_.c_str();
            v.kind = JsonValue::Number;
        }
        return v;
    }
};

// ---- YAML (block style) ------------------------------------------------------------
// The reference reads its config with YAML::LoadFile (src/ConfigParserYAML.cpp:12), so a
// config may be a JSON document (YAML's flow style; the shipped config.json) or block
// YAML.  This reader covers the block subset a config uses: nested mappings and "- "
// sequences by indentation, inline flow collections ([..], {..}, possibly spanning
// lines), quoted and plain scalars, '#' comments.  Plain scalars are typed the way the
// parser's .as<T>() calls read them: numbers, YAML 1.1 booleans, null / ~, else strings
// (a number keeps its text, for .as<std::string>()).  Anchors, tags, multi-document
// streams and block scalars (| >) are not supported and raise.
class YamlReader {
public:
    explicit YamlReader(const std::string& text) {
        std::istringstream in(text);
        std::string raw;
        int no = 0;
        while (std::getline(in, raw)) {
            ++no;
            if (!raw.empty() && raw.back() == '\r') raw.pop_back();
            const std::string s = strip_comment(raw);
            size_t ind = 0;
            while (ind < s.size() && s[ind] == ' ') ++ind;
            if (ind < s.size() && s[ind] == '\t') fail(no, "tab indentation");
            std::string body = trim(s.substr(ind));
            if (body.empty()) continue;
            if (body == "---" && lines_.empty()) continue;
            if (body == "---" || body == "...") fail(no, "multi-document streams are not supported");
            lines_.push_back({(int)ind, body, no});
        }
    }
    JsonValue parse() {
        if (lines_.empty()) return JsonValue();
        JsonValue v = block(lines_[0].indent);
        if (i_ != lines_.size()) fail(lines_[i_].no, "bad indentation");
        return v;
    }

private:
    struct Line {
        int indent;
        std::string body;
        int no;
    };
    std::vector<Line> lines_;
    size_t i_ = 0;

    [[noreturn]] static void fail(int no, const std::string& m) {
        throw std::runtime_error("config YAML parse error at line " + std::to_string(no) + ": " + m);
    }
    static std::string trim(const std::string& s) {
        size_t a = 0, b = s.size();
        while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
        while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
        return s.substr(a, b - a);
    }
    // drops a comment: '#' at the start or after a blank, outside quotes
    static std::string strip_comment(const std::string& s) {
        char q = 0;
        for (size_t k = 0; k < s.size(); ++k) {
            const char c = s[k];
            if (q) {
                if (c == q) q = 0;
                else if (c == '\\' && q == '"') ++k;
            } else if (c == '"' || c == '\'') {
                q = c;
            } else if (c == '#' && (k == 0 || s[k - 1] == ' ' || s[k - 1] == '\t')) {
                return s.substr(0, k);
            }
        }
        return s;
    }
    static bool is_seq_item(const std::string& b) { return b == "-" || b.rfind("- ", 0) == 0; }
    // position of the ':' that ends a mapping key (followed by a blank or the line end), or npos
    static size_t key_colon(const std::string& b) {
        if (b.empty() || b[0] == '[' || b[0] == '{') return std::string::npos;
        char q = 0;
        size_t k = 0;
        if (b[0] == '"' || b[0] == '\'') {
            q = b[0];
            for (k = 1; k < b.size() && b[k] != q; ++k)
                if (b[k] == '\\' && q == '"') ++k;
            ++k;
        }
        for (; k < b.size(); ++k)
            if (b[k] == ':' && (k + 1 == b.size() || b[k + 1] == ' ')) return k;
        return std::string::npos;
    }
    static std::string unquote_key(const std::string& k, int no) {
        if (k.size() >= 2 && (k[0] == '"' || k[0] == '\'')) {
            JsonValue v = scalar(k, no);
            return v.str;
        }
        return k;
    }
    // a plain or quoted scalar, typed
    static JsonValue scalar(const std::string& t, int no) {
        JsonValue v;
        if (t.empty()) return v;  // null
        if (t[0] == '"' || t[0] == '\'') {
            const char q = t[0];
            std::string out;
            size_t k = 1;
            for (; k < t.size(); ++k) {
                char c = t[k];
                if (c == q) {
                    if (q == '\'' && k + 1 < t.size() && t[k + 1] == '\'') {
                        out += '\'';
                        ++k;
                        continue;
                    }
                    break;
                }
                if (q == '"' && c == '\\' && k + 1 < t.size()) {
                    c = t[++k];
                    out += c == 'n' ? '\n' : c == 't' ? '\t' : c;
                    continue;
                }
                out += c;
            }
            if (k >= t.size() || trim(t.substr(k + 1)) != "") fail(no, "bad quoted scalar " + t);
            v.kind = JsonValue::String;
            v.str = out;
            return v;
        }
        if (t[0] == '&' || t[0] == '*' || t[0] == '!' || t[0] == '|' || t[0] == '>')
            fail(no, "anchors, aliases, tags and block scalars are not supported");
        if (t == "~" || t == "null" || t == "Null" || t == "NULL") return v;
        static const char* yes[] = {"true", "True", "TRUE", "yes", "Yes", "YES", "on", "On", "ON", "y", "Y"};
        static const char* no_[] = {"false", "False", "FALSE", "no", "No", "NO", "off", "Off", "OFF", "n", "N"};
        // Bool and Number scalars keep their text: yaml-cpp's .as<std::string>() returns it
        v.str = t;
        for (const char* s : yes)
            if (t == s) {
                v.kind = JsonValue::Bool;
                v.b = true;
                return v;
            }
        for (const char* s : no_)
            if (t == s) {
                v.kind = JsonValue::Bool;
                v.b = false;
                return v;
            }
        double d = 0.0;
        if (yaml_number(t, d)) {
            v.kind = JsonValue::Number;
            v.num = d;
            return v;
        }
        v.kind = JsonValue::String;
        return v;
    }
    // A plain scalar yaml-cpp's .as<double>() reads: decimal [-+]?(digits[.digits]|.digits)
    // with an optional exponent, or [-+]?.inf / .nan (any of the three spellings).  Text
    // strtod alone would also take (nan, inf, hex, ...) stays a string.
    static bool yaml_number(const std::string& t, double& out) {
        size_t k = 0;
        const bool neg = k < t.size() && t[k] == '-';
        if (k < t.size() && (t[k] == '-' || t[k] == '+')) ++k;
        const std::string rest = t.substr(k);
        if (rest == ".inf" || rest == ".Inf" || rest == ".INF") {
            out = neg ? -HUGE_VAL : HUGE_VAL;
            return true;
        }
        if (k == 0 && (rest == ".nan" || rest == ".NaN" || rest == ".NAN")) {
            out = std::nan("");
            return true;
        }
        size_t digits = 0;
        while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k, ++digits;
        if (k < t.size() && t[k] == '.') {
            ++k;
            while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k, ++digits;
        }
        if (digits == 0) return false;
        if (k < t.size() && (t[k] == 'e' || t[k] == 'E')) {
            ++k;
            if (k < t.size() && (t[k] == '-' || t[k] == '+')) ++k;
            size_t ed = 0;
            while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k, ++ed;
            if (ed == 0) return false;
        }
        if (k != t.size()) return false;
        out = std::strtod(t.c_str(), nullptr);
        return true;
    }
    // flow collection text -> value; plain scalars inside are typed as above
    static JsonValue flow(const std::string& t, int no) {
        size_t k = 0;
        JsonValue v = flow_value(t, k, no);
        while (k < t.size() && t[k] == ' ') ++k;
        if (k != t.size()) fail(no, "trailing characters after a flow collection");
        return v;
    }
    static JsonValue flow_value(const std::string& t, size_t& k, int no) {
        while (k < t.size() && t[k] == ' ') ++k;
        if (k >= t.size()) fail(no, "unexpected end of a flow collection");
        JsonValue v;
        const char c = t[k];
        if (c == '[' || c == '{') {
            const bool map = c == '{';
            v.kind = map ? JsonValue::Object : JsonValue::Array;
            ++k;
            while (true) {
                while (k < t.size() && t[k] == ' ') ++k;
                if (k < t.size() && t[k] == (map ? '}' : ']')) {
                    ++k;
                    return v;
                }
                if (map) {
                    const size_t a = k;
                    JsonValue key = flow_value(t, k, no);
                    while (k < t.size() && t[k] == ' ') ++k;
                    if (k >= t.size() || t[k] != ':') fail(no, "expected ':' in a flow mapping");
                    ++k;
                    std::string ks = key.kind == JsonValue::String || key.kind == JsonValue::Number
                                         ? key.str
                                         : trim(t.substr(a, k - 1 - a));
                    v.obj.emplace_back(ks, flow_value(t, k, no));
                } else {
                    v.arr.push_back(flow_value(t, k, no));
                }
                while (k < t.size() && t[k] == ' ') ++k;
                if (k < t.size() && t[k] == ',') {
                    ++k;
                    continue;
                }
                if (k < t.size() && t[k] == (map ? '}' : ']')) {
                    ++k;
                    return v;
                }
                fail(no, "expected ',' or a closing bracket");
            }
        }
        // a scalar: quoted, or plain up to the next , ] } (or ':' + blank in a mapping)
        const size_t a = k;
        if (c == '"' || c == '\'') {
            ++k;
            while (k < t.size() && t[k] != c) k += (t[k] == '\\' && c == '"') ? 2 : 1;
            ++k;
        } else {
            while (k < t.size() && t[k] != ',' && t[k] != ']' && t[k] != '}' &&
                   !(t[k] == ':' && (k + 1 == t.size() || t[k + 1] == ' ')))
                ++k;
        }
        return scalar(trim(t.substr(a, k - a)), no);
    }
    // a value written after "key:" or "- " on line `no`: flow collections may continue on
    // the following lines until their brackets balance
    JsonValue inline_value(std::string t, int no) {
        if (!t.empty() && (t[0] == '[' || t[0] == '{')) {
            auto depth = [](const std::string& s) {
                int d = 0;
                char q = 0;
                for (size_t k = 0; k < s.size(); ++k) {
                    const char c = s[k];
                    if (q) {
                        if (c == q) q = 0;
                    } else if (c == '"' || c == '\'') {
                        q = c;
                    } else if (c == '[' || c == '{') {
                        ++d;
                    } else if (c == ']' || c == '}') {
                        --d;
                    }
                }
                return d;
            };
            while (depth(t) > 0) {
                if (i_ >= lines_.size()) fail(no, "unterminated flow collection");
                t += " " + lines_[i_++].body;
            }
            return flow(t, no);
        }
        return scalar(t, no);
    }
    JsonValue block(int indent) {
        if (i_ >= lines_.size()) return JsonValue();
        return is_seq_item(lines_[i_].body) ? sequence(indent) : mapping(indent);
    }
    // the value of a "key:" / "- " with nothing after it: the more-indented block below
    // (a sequence may sit at the key's own indentation), else null
    JsonValue nested(int indent, bool seq_same_level) {
        if (i_ < lines_.size()) {
            const Line& n = lines_[i_];
            if (n.indent > indent) return block(n.indent);
            if (seq_same_level && n.indent == indent && is_seq_item(n.body)) return sequence(indent);
        }
        return JsonValue();
    }
    JsonValue mapping(int indent) {
        JsonValue v;
        v.kind = JsonValue::Object;
        while (i_ < lines_.size() && lines_[i_].indent == indent && !is_seq_item(lines_[i_].body)) {
            const Line ln = lines_[i_++];
            const size_t c = key_colon(ln.body);
            if (c == std::string::npos) {
                if (v.obj.empty() && ln.body[0] != '[' && ln.body[0] != '{') fail(ln.no, "expected 'key: value'");
                if (!v.obj.empty()) fail(ln.no, "expected 'key: value'");
                --i_;  // a document that is a single flow collection / scalar
                const Line one = lines_[i_++];
                return inline_value(one.body, one.no);
            }
            const std::string key = unquote_key(trim(ln.body.substr(0, c)), ln.no);
            const std::string rest = trim(ln.body.substr(c + 1));
            for (const auto& kv : v.obj)
                if (kv.first == key) fail(ln.no, "duplicate key " + key);
            v.obj.emplace_back(key, rest.empty() ? nested(indent, true) : inline_value(rest, ln.no));
        }
        if (i_ < lines_.size() && lines_[i_].indent > indent) fail(lines_[i_].no, "bad indentation");
        return v;
    }
    JsonValue sequence(int indent) {
        JsonValue v;
        v.kind = JsonValue::Array;
        while (i_ < lines_.size() && lines_[i_].indent == indent && is_seq_item(lines_[i_].body)) {
            Line& ln = lines_[i_];
            const std::string rest = ln.body == "-" ? std::string() : trim(ln.body.substr(2));
            if (rest.empty()) {
                ++i_;
                v.arr.push_back(nested(indent, false));
            } else if (key_colon(rest) != std::string::npos || is_seq_item(rest)) {
                // "- key: value" / "- - x": a nested block starting on this line
                const int inner = indent + (int)(ln.body.size() - rest.size());
                ln.indent = inner;
                ln.body = rest;
                v.arr.push_back(block(inner));
            } else {
                ++i_;
                v.arr.push_back(inline_value(rest, ln.no));
            }
        }
        return v;
    }
};

// A document whose first significant character opens a JSON object or array is read as
// JSON (the shipped config.json), anything else as block YAML.
JsonValue parse_config_text(const std::string& text) {
    size_t k = 0;
    while (k < text.size()) {
        const char c = text[k];
        if (c == ' ' || c == '\t' || c == '\r' || c == '\n') {
            ++k;
        } else if (c == '#') {
            while (k < text.size() && text[k] != '\n') ++k;
        } else {
            break;
        }
    }
    if (k < text.size() && (text[k] == '{' || text[k] == '[')) {
        try {
            return Reader(text).parse();
        } catch (const std::runtime_error&) {
            try {
                return YamlReader(text).parse();  // flow YAML that is not strict JSON
            } catch (const std::runtime_error&) {
            }
            throw;  // report the JSON error
        }
    }
    return YamlReader(text).parse();
}

const JsonValue& at(const JsonValue& v, const std::string& k, const std::string& path) {
    const JsonValue* r = v.kind == JsonValue::Object ? v.find(k) : nullptr;
    if (!r) throw std::runtime_error("config: missing key " + path + k);
    return *r;
}
double num(const JsonValue& v, const std::string& what) {
    if (v.kind == JsonValue::Number) return v.num;
    if (v.kind == JsonValue::Bool) return v.b ? 1.0 : 0.0;
    throw std::runtime_error("config: " + what + " is not a number");
}
bool boolean(const JsonValue& v, const std::string& what) {
    if (v.kind == JsonValue::Bool) return v.b;
    if (v.kind == JsonValue::Number) return v.num != 0;
    if (v.kind == JsonValue::String) return v.str == "true" || v.str == "True" || v.str == "1";
    throw std::runtime_error("config: " + what + " is not a bool");
}
std::string str(const JsonValue& v, const std::string& what) {
    if (v.kind == JsonValue::String) return v.str;
    if ((v.kind == JsonValue::Number || v.kind == JsonValue::Bool) && !v.str.empty()) return v.str;  // YAML plain scalar
    throw std::runtime_error("config: " + what + " is not a string");
}
Vec3 vec3(const JsonValue& v, const std::string& what) {
    if (v.kind != JsonValue::Array || v.arr.size() < 3) throw std::runtime_error("config: " + what + " is not a 3-vector");
    return {num(v.arr[0], what), num(v.arr[1], what), num(v.arr[2], what)};
}

}  // namespace

ConfigParser::ConfigParser(const std::string& configPath) {
    std::ifstream f(configPath);
    if (!f) throw std::runtime_error("bad file: " + configPath);  // YAML::BadFile
    std::stringstream ss;
    ss << f.rdbuf();
    parse(parse_config_text(ss.str()));
}

std::shared_ptr<ConfigParser> ConfigParser::fromString(const std::string& json) {
    std::shared_ptr<ConfigParser> p(new ConfigParser());
    p->parse(parse_config_text(json));
    return p;
}

void ConfigParser::parse(const JsonValue& root) {
    // parseGeometries — src/ConfigParserYAML.cpp:54-73 (half size = size / 2)
    const JsonValue& geo = at(root, "component_geometry", "");
    for (const auto& comp : geo.obj) {
        std::vector<OBBDescription> descs;
        for (const auto& o : comp.second.obj) {
            const std::string p = "component_geometry." + comp.first + "." + o.first + ".";
            OBBDescription d;
            d.center = vec3(at(o.second, "position", p), p + "position");
            d.halfSize = vec3(at(o.second, "size", p), p + "size") / 2;
            d.type = str(at(o.second, "type", p), p + "type");
            const JsonValue* nm = o.second.find("name");  // required by the reference (:65)
            d.name = nm ? str(*nm, p + "name") : o.first;
            if (d.type != "collision" && d.type != "filling")
                throw std::runtime_error("config: unknown OBB type " + d.type);
            descs.push_back(d);
        }
        objects[comp.first] = descs;
    }
    // parseObjectProperties — :75-83
    for (const auto& o : at(root, "component_properties", "").obj)
        objectProperties[o.first] = {num(at(o.second, "height", "component_properties." + o.first + "."), "height")};
    // gate_id_to_name_mapping — :21-32
    const JsonValue& map = at(root, "gate_id_to_name_mapping", "");
    gateTypeNames.assign(map.obj.size(), "");
    for (const auto& kv : map.obj) {
        const int id = std::atoi(kv.first.c_str());
        if (id < 0 || id >= (int)map.obj.size()) throw std::runtime_error("config: gate ids must be 0..n-1");
        gateTypeNames[id] = str(kv.second, "gate_id_to_name_mapping");
    }
    // parseWorldProperties — :85-92
    const JsonValue& wp = at(root, "world_properties", "");
    world.lowerBound = vec3(at(wp, "lower_bound", "world_properties."), "lower_bound");
    world.upperBound = vec3(at(wp, "upper_bound", "world_properties."), "upper_bound");
    const JsonValue& ir = at(wp, "inflate_radius", "world_properties.");
    world.inflateRadius["gate"] = num(at(ir, "gate", "world_properties.inflate_radius."), "gate");
    world.inflateRadius["obstacle"] = num(at(ir, "obstacle", "world_properties.inflate_radius."), "obstacle");
    // parsePathPlannerProperties — :94-108
    const JsonValue& pp = at(root, "path_planner_properties", "");
    const std::string ppn = "path_planner_properties.";
    pathPlanner.optimalityThresholdPercentage = num(at(pp, "optimality_threshold_percentage", ppn), "x");
    pathPlanner.timeLimitOnline = num(at(pp, "time_limit_online", ppn), "time_limit_online");
    pathPlanner.timeLimitOffline = num(at(pp, "time_limit_offline", ppn), "time_limit_offline");
    pathPlanner.checkpointGateOffset = num(at(pp, "checkpoint_gate_offset", ppn), "checkpoint_gate_offset");
    pathPlanner.range = num(at(pp, "range", ppn), "range");
    pathPlanner.minDistCheckTrajCollision = num(at(pp, "min_dist_check_traj_collision", ppn), "x");
    pathPlanner.pathSimplification = str(at(pp, "path_simplification", ppn), "path_simplification");
    pathPlanner.recalculateOnline = boolean(at(pp, "recalculate_online", ppn), "recalculate_online");
    pathPlanner.canPassGate = boolean(at(pp, "can_pass_gate", ppn), "can_pass_gate");
    pathPlanner.advanceForCalculation = boolean(at(pp, "advance_for_calculation", ppn), "x");
    pathPlanner.planner = str(at(pp, "planner", ppn), "planner");
    pathPlanner.samplesFMT = (int)num(at(pp, "samples_fmt", ppn), "samples_fmt");
    // parseTrajectoryGeneratorProperties — :110-118
    const JsonValue& tg = at(root, "trajectory_generator_properties", "");
    const std::string tgn = "trajectory_generator_properties.";
    trajectoryGenerator.maxVelocity = num(at(tg, "max_velocity", tgn), "max_velocity");
    trajectoryGenerator.maxAcceleration = num(at(tg, "max_acceleration", tgn), "max_acceleration");
    trajectoryGenerator.samplingInterval = num(at(tg, "sampling_interval", tgn), "sampling_interval");
    trajectoryGenerator.type = str(at(tg, "type", tgn), "type");
    trajectoryGenerator.maxTime = num(at(tg, "max_time", tgn), "max_time");
    trajectoryGenerator.prependTrajTime = num(at(tg, "prepend_traj_time", tgn), "prepend_traj_time");
    trajectoryGenerator.maxTrajDivergence = num(at(tg, "max_traj_divergence", tgn), "max_traj_divergence");
}

const std::vector<OBBDescription>& ConfigParser::getGateGeometryByTypeId(int typeId) const {
    if (typeId < 0 || typeId >= (int)gateTypeNames.size())
        throw std::runtime_error("config: unknown gate type id " + std::to_string(typeId));
    return objects.at(gateTypeNames[typeId]);
}
const std::vector<OBBDescription>& ConfigParser::getObstacleGeometry() const { return objects.at("obstacle"); }
const ObjectProperties& ConfigParser::getObjectPropertiesByTypeId(int typeId) const {
    if (typeId < 0 || typeId >= (int)gateTypeNames.size())
        throw std::runtime_error("config: unknown gate type id " + std::to_string(typeId));
    return objectProperties.at(gateTypeNames[typeId]);
}
const WorldProperties& ConfigParser::getWorldProperties() const { return world; }
const PathPlannerProperties& ConfigParser::getPathPlannerProperties() const { return pathPlanner; }
const TrajectoryGeneratorProperties& ConfigParser::getTrajectoryGeneratorProperties() const {
    return trajectoryGenerator;
}

}  // namespace epp
