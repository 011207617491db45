// epp/ConfigParser.h — planner configuration, drop-in for the reference's ConfigParser
// (include/ConfigParserYAML.h, src/ConfigParserYAML.cpp:10-118) and its structs
// (include/Types.h:21-79).  Reads JSON (the format of the reference's shipped
// config.json; yaml-cpp is not a dependency of this build).  Missing keys throw
// std::runtime_error naming the key, as yaml-cpp's as<T>() would throw.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "epp/types.h"

namespace epp {

struct OBBDescription {  // include/Types.h:21-27
    Vec3 center;
    Vec3 halfSize;
    std::string type;  // "collision" | "filling"
    std::string name;
};

struct ObjectProperties {  // include/Types.h:32-35
    double height = 0;
};

struct WorldProperties {  // include/Types.h:40-45
    Vec3 lowerBound;
    Vec3 upperBound;
    std::map<std::string, double> inflateRadius;
};

struct PathPlannerProperties {  // include/Types.h:50-64
    double optimalityThresholdPercentage = 0;
    double timeLimitOnline = 0;
    double timeLimitOffline = 0;
    double checkpointGateOffset = 0;
    double range = 0;
    double minDistCheckTrajCollision = 0;
    std::string pathSimplification;
    bool recalculateOnline = false;
    bool advanceForCalculation = false;
    bool canPassGate = false;
    std::string planner;
    int samplesFMT = 0;
};

struct TrajectoryGeneratorProperties {  // include/Types.h:69-79
    double maxVelocity = 0;
    double maxAcceleration = 0;
    double samplingInterval = 0;
    std::string type;
    double maxTime = 0;
    double maxTrajDivergence = 0;
    double prependTrajTime = 0;
};

class JsonValue;  // minimal order-preserving JSON DOM (host_config.cpp)

class ConfigParser {
public:
    explicit ConfigParser(const std::string& configPath);
    // Parses a JSON document held in memory.
    static std::shared_ptr<ConfigParser> fromString(const std::string& json);

    const std::vector<OBBDescription>& getGateGeometryByTypeId(int typeId) const;
    const std::vector<OBBDescription>& getObstacleGeometry() const;
    const ObjectProperties& getObjectPropertiesByTypeId(int typeId) const;
    const WorldProperties& getWorldProperties() const;
    const PathPlannerProperties& getPathPlannerProperties() const;
    const TrajectoryGeneratorProperties& getTrajectoryGeneratorProperties() const;
    int numGateTypes() const { return (int)gateTypeNames.size(); }

    // mutable access for programmatic configuration (tests, benches)
    PathPlannerProperties& pathPlannerProperties() { return pathPlanner; }
    TrajectoryGeneratorProperties& trajectoryGeneratorProperties() { return trajectoryGenerator; }

private:
    ConfigParser() = default;
    void parse(const JsonValue& root);
    std::map<std::string, std::vector<OBBDescription>> objects;
    std::map<std::string, ObjectProperties> objectProperties;
    std::vector<std::string> gateTypeNames;  // gate_id_to_name_mapping, by type id
    WorldProperties world;
    PathPlannerProperties pathPlanner;
    TrajectoryGeneratorProperties trajectoryGenerator;
};

}  // namespace epp
