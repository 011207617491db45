// host_config.cpp — ConfigParser (src/ConfigParserYAML.cpp:10-118) over a small
// order-preserving JSON reader.  Object members keep document order, which is the
// iteration order yaml-cpp gives the reference for component_geometry.
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
        } else if (lit("false")) {
            v.kind = JsonValue::Bool;
            v.b = false;
        } else if (lit("null")) {
            v.kind = JsonValue::Null;
        } else {
            char* end = nullptr;
            v.num = std::strtod(s_.c_str() + i_, &end);
            if (end == s_.c_str() + i_) fail("bad value");
            i_ = end - s_.c_str();
            v.kind = JsonValue::Number;
        }
        return v;
    }
};

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
    const std::string text = ss.str();
    parse(Reader(text).parse());
}

std::shared_ptr<ConfigParser> ConfigParser::fromString(const std::string& json) {
    std::shared_ptr<ConfigParser> p(new ConfigParser());
    p->parse(Reader(json).parse());
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
