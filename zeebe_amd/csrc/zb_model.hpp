// zb_model.hpp — deployment-time compiler: BPMN XML -> flat device tables (zb_device.hpp).
//
// Follows the reference transformer's observable semantics:
//   - two walks over the DOM, siblings visited last-to-first (ModelWalker.java:53-69), so every
//     node's executable outgoing list is in reverse document order (SequenceFlowHandler.java:82);
//   - lifecycle bindings per element type, supertype handlers first (BpmnTransformer.java:52-83,
//     handler/*.java; TypeHierarchyVisitor.java:34-41);
//   - exclusive gateway binds EXCLUSIVE_SPLIT iff its first model-order <outgoing> flow has a
//     condition (ExclusiveGatewayHandler.java:49-63);
//   - json-el conditions compiled to a jump program over json-path queries
//     (JsonConditionParser.scala:53-114, JsonPathQueryCompiler.java:51-125).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "zb_device.hpp"

namespace zbg {

struct ModelTables {
  std::vector<DevElem> elems;
  std::vector<DevWorkflow> workflows;
  std::vector<uint16_t> cond_flows;
  std::vector<uint32_t> code;
  std::vector<DevConst> consts;
  std::vector<DevQuery> queries;
  std::vector<DevFilter> filters;
  std::vector<uint8_t> pool;
  std::vector<DevMapping> maps;  // explicit io-mappings (DevElem.map_in / map_out ranges)
  std::vector<DevSeg> segs;      // their target path segments
  // host-only
  std::vector<std::string> elem_ids;

  uint32_t add_bytes(const std::string& s);
  std::string str(uint32_t off, uint32_t len) const {
    return std::string((const char*)pool.data() + off, len);
  }
};

// Deploys every process of the resource. Returns 0 or ZB_EDEPLOY / ZB_EUNSUPPORTED with msg.
int compile_deployment(ModelTables& t, const std::string& xml, int64_t workflow_key, int32_t version,
                       std::string& err);

// json-path compilation into t.queries/t.filters; returns query index or -1 (invalid, err set)
int compile_query(ModelTables& t, const std::string& expr, std::string& err);

// one io-mapping (Mapping.java): the source compiled as a json-path query, the target split into the
// LITERAL / ROOT_OBJECT tokens of JsonPathTokenizer (MsgPackDocumentExtractor.extract walks them); appended
// to t.maps / t.segs, returns its index or -1 (err set)
int compile_mapping(ModelTables& t, const std::string& source, const std::string& target, std::string& err);

// json-el compilation; returns program offset in t.code or -1 (err set)
int compile_condition(ModelTables& t, const std::string& expr, std::string& err);

}  // namespace zbg
