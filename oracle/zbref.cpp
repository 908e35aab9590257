// zbref — ORACLE / TEST INFRASTRUCTURE ONLY.
//
// A sequential CPU restatement of the reference's workflow-instance stepping path (Zeebe
// 0.12.0-SNAPSHOT broker-core). It exists to *check* the product (libzbgpu.so) and to give the
// CPU baseline timed by bench.py; it is never called by the product. Parity is pinned by the
// reference's own known-answer tests transcribed under tests/golden (see tests/test_oracle_*.py).
//
// What it restates (file:line in /root/reference):
//   FIFO driver              logstreams/src/main/java/io/zeebe/logstreams/processor/StreamProcessorController.java:296-414
//   processor registrations  broker-core/src/main/java/io/zeebe/broker/workflow/processor/WorkflowInstanceStreamProcessor.java:90-182
//   CREATE/CREATED/JOB/CORRELATE/CANCEL/UPDATE_PAYLOAD       same file :224-576
//   step dispatch + guards   broker-core/.../workflow/processor/BpmnStepProcessor.java:92-251
//   step handlers            broker-core/.../workflow/processor/{activity,catchevent,exclusivegw,flownode,process,
//                            sequenceflow,servicetask,subprocess}/*.java
//   index writes             broker-core/.../workflow/processor/ElementInstanceWriter.java:64-110
//   element instance index   broker-core/.../workflow/index/{ElementInstance,ElementInstanceIndex}.java
//   key generator            broker-core/.../logstreams/processor/KeyGenerator.java:28-72
//   typed writers            broker-core/.../logstreams/processor/TypedCommandWriterImpl.java:85-143,
//                            TypedStreamWriterImpl.java:44-152 (a non-batch writer keeps only its last record)
//   transformer              broker-core/.../workflow/model/transformation/** + bpmn-model/.../traversal/ModelWalker.java:53-69
//   record values            broker-core/.../workflow/data/WorkflowInstanceRecord.java:39-60,
//                            broker-core/.../job/data/{JobRecord,JobHeaders}.java, broker-core/.../incident/data/IncidentRecord.java
//   canonical job harness    broker-core/src/test/java/io/zeebe/broker/util/TestStreams.java:112-142 and
//                            broker-core/src/test/.../workflow/processor/WorkflowInstanceStreamProcessorTest.java:206-211
//                            (JOB CREATE command at its FIFO position -> JOB CREATED(k), JOB COMPLETED(k); job keys
//                            from KeyGenerator(2, 5))
// Positions are log sequence numbers (0-based record index); byte positions of the real log are out of scope.
#include <malloc.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "zbref_el.hpp"
#include "zbref_mapping.hpp"
#include "zbref_xml.hpp"

namespace zbref {

// ------------------------------------------------------------------------------ protocol enums
enum ValueType : uint8_t { VT_JOB = 0, VT_WORKFLOW_INSTANCE = 5, VT_INCIDENT = 6, VT_MESSAGE = 10,
                           VT_MESSAGE_SUBSCRIPTION = 11, VT_WORKFLOW_INSTANCE_SUBSCRIPTION = 12 };
enum RecordType : uint8_t { RT_EVENT = 0, RT_COMMAND = 1, RT_REJECTION = 2 };
enum WfIntent : uint8_t {
  CREATE = 0, CREATED = 1, START_EVENT_OCCURRED = 2, END_EVENT_OCCURRED = 3, SEQUENCE_FLOW_TAKEN = 4,
  GATEWAY_ACTIVATED = 5, ELEMENT_READY = 6, ELEMENT_ACTIVATED = 7, ELEMENT_COMPLETING = 8, ELEMENT_COMPLETED = 9,
  ELEMENT_TERMINATING = 10, ELEMENT_TERMINATED = 11, CANCEL = 12, CANCELING = 13, UPDATE_PAYLOAD = 14,
  PAYLOAD_UPDATED = 15
};
enum JobIntentE : uint8_t { JOB_CREATE = 0, JOB_CREATED = 1, JOB_ACTIVATE = 2, JOB_ACTIVATED = 3, JOB_COMPLETE = 4,
                            JOB_COMPLETED = 5, JOB_TIME_OUT = 6, JOB_TIMED_OUT = 7, JOB_FAIL = 8, JOB_FAILED = 9,
                            JOB_UPDATE_RETRIES = 10, JOB_RETRIES_UPDATED = 11, JOB_CANCEL = 12, JOB_CANCELED = 13 };
enum IncidentIntentE : uint8_t { INCIDENT_CREATE = 0 };
enum WisIntent : uint8_t { WIS_CORRELATE = 0, WIS_CORRELATED = 1 };  // WorkflowInstanceSubscriptionIntent.java:19-20
enum MsgIntent : uint8_t { MSG_PUBLISH = 0, MSG_PUBLISHED = 1, MSG_DELETE = 2, MSG_DELETED = 3 };  // MessageIntent.java:19-23
enum MsgSubIntent : uint8_t { MSUB_OPEN = 0, MSUB_OPENED = 1 };  // MessageSubscriptionIntent.java:19-20
enum RejectionTypeE : uint8_t { REJ_BAD_VALUE = 0, REJ_NOT_APPLICABLE = 1, REJ_PROCESSING_ERROR = 2, REJ_NULL = 255 };
enum ErrorTypeE : uint8_t { ERR_UNKNOWN = 0, ERR_IO_MAPPING = 1, ERR_JOB_NO_RETRIES = 2, ERR_CONDITION = 3 };

static const char* ERROR_TYPE_NAMES[] = {"UNKNOWN", "IO_MAPPING_ERROR", "JOB_NO_RETRIES", "CONDITION_ERROR"};

// BpmnStep.java:20-54
enum Step : uint8_t {
  S_NONE = 0, S_TAKE_SEQUENCE_FLOW, S_CONSUME_TOKEN, S_EXCLUSIVE_SPLIT, S_CREATE_JOB, S_APPLY_INPUT_MAPPING,
  S_APPLY_OUTPUT_MAPPING, S_ACTIVATE_GATEWAY, S_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE, S_START_STATEFUL_ELEMENT,
  S_TRIGGER_END_EVENT, S_TRIGGER_START_EVENT, S_TERMINATE_CONTAINED_INSTANCES, S_TERMINATE_JOB_TASK,
  S_TERMINATE_ELEMENT, S_PROPAGATE_TERMINATION, S_CANCEL_PROCESS, S_COMPLETE_PROCESS,
  // EXTENSION (parity unpinned): the reference rejects parallel gateways at deployment
  // (bpmn-model/.../validation/zeebe/FlowElementValidator.java:36-58); DESIGN.md §C4 defines these two.
  S_PARALLEL_SPLIT, S_PARALLEL_MERGE,
  S_UNBOUND = 255
};

static const bytes EMPTY_DOCUMENT = bytes("\x80", 1);

// ------------------------------------------------------------------------------ record values
struct WfValue {  // WorkflowInstanceRecord.java:39-60
  bytes bpmn_process_id;
  int32_t version = -1;
  int64_t workflow_key = -1;
  int64_t workflow_instance_key = -1;
  bytes activity_id;
  bytes payload = EMPTY_DOCUMENT;
  int64_t scope_instance_key = -1;
  void set_payload(const bytes& p) {  // DocumentValue.wrap: nil / empty -> {}
    if (p.empty() || (p.size() == 1 && (uint8_t)p[0] == 0xc0)) payload = EMPTY_DOCUMENT;
    else {
      if (mp_format_type((uint8_t)p[0]) != MpType::MAP)
        throw ZbError("Document has invalid format. On root level an object is only allowed.");
      payload = p;
    }
  }
  bytes encode() const {
    MpWriter w;
    w.map_header(7);
    w.str("bpmnProcessId"); w.str(bpmn_process_id);
    w.str("version"); w.integer(version);
    w.str("workflowKey"); w.integer(workflow_key);
    w.str("workflowInstanceKey"); w.integer(workflow_instance_key);
    w.str("activityId"); w.str(activity_id);
    w.str("payload"); w.bin(payload);
    w.str("scopeInstanceKey"); w.integer(scope_instance_key);
    return w.b;
  }
};

struct JobValue {  // JobRecord.java:35-53 + JobHeaders.java:33-51
  int64_t deadline = INT64_MIN;  // Protocol.INSTANT_NULL_VALUE
  bytes worker;
  int32_t retries = -1;
  bytes type;
  bytes h_bpmn_process_id;
  int32_t h_version = -1;
  int64_t h_workflow_key = -1;
  int64_t h_workflow_instance_key = -1;
  bytes h_activity_id;
  int64_t h_activity_instance_key = -1;
  bytes custom_headers = EMPTY_DOCUMENT;  // PackedProperty, written raw
  bytes payload = EMPTY_DOCUMENT;
  bytes encode() const {
    MpWriter w;
    w.map_header(7);
    w.str("deadline"); w.integer(deadline);
    w.str("worker"); w.str(worker);
    w.str("retries"); w.integer(retries);
    w.str("type"); w.str(type);
    w.str("headers");
    w.map_header(6);
    w.str("bpmnProcessId"); w.str(h_bpmn_process_id);
    w.str("workflowDefinitionVersion"); w.integer(h_version);
    w.str("workflowKey"); w.integer(h_workflow_key);
    w.str("workflowInstanceKey"); w.integer(h_workflow_instance_key);
    w.str("activityId"); w.str(h_activity_id);
    w.str("activityInstanceKey"); w.integer(h_activity_instance_key);
    w.str("customHeaders"); w.raw(custom_headers);
    w.str("payload"); w.bin(payload);
    return w.b;
  }
};

struct IncidentValue {  // IncidentRecord.java
  uint8_t error_type = ERR_UNKNOWN;
  bytes error_message;
  int64_t failure_event_position = -1;
  bytes bpmn_process_id;
  int64_t workflow_instance_key = -1;
  bytes activity_id;
  int64_t activity_instance_key = -1;
  int64_t job_key = -1;
  bytes payload = EMPTY_DOCUMENT;
  bytes encode() const {
    MpWriter w;
    w.map_header(9);
    w.str("errorType"); w.str(ERROR_TYPE_NAMES[error_type]);
    w.str("errorMessage"); w.str(error_message);
    w.str("failureEventPosition"); w.integer(failure_event_position);
    w.str("bpmnProcessId"); w.str(bpmn_process_id);
    w.str("workflowInstanceKey"); w.integer(workflow_instance_key);
    w.str("activityId"); w.str(activity_id);
    w.str("activityInstanceKey"); w.integer(activity_instance_key);
    w.str("jobKey"); w.integer(job_key);
    w.str("payload"); w.bin(payload);
    return w.b;
  }
};

// WorkflowInstanceSubscriptionRecord.java:26-38: four properties, no partition id (pinned by
// IntermediateMessageCatchEventTest.java:357-362, containsExactly)
struct WisValue {
  int64_t workflow_instance_key = -1;
  int64_t activity_instance_key = -1;
  bytes message_name;
  bytes payload = EMPTY_DOCUMENT;
  bytes encode() const {
    MpWriter w;
    w.map_header(4);
    w.str("workflowInstanceKey"); w.integer(workflow_instance_key);
    w.str("activityInstanceKey"); w.integer(activity_instance_key);
    w.str("messageName"); w.str(message_name);
    w.str("payload"); w.bin(payload);
    return w.b;
  }
};

// MessageSubscriptionRecord.java:26-41 (pinned by IntermediateMessageCatchEventTest.java:132-138)
struct MsgSubValue {
  int32_t wf_partition = 0;
  int64_t workflow_instance_key = -1;
  int64_t activity_instance_key = -1;
  bytes message_name;
  bytes correlation_key;
  bytes encode() const {
    MpWriter w;
    w.map_header(5);
    w.str("workflowInstancePartitionId"); w.integer(wf_partition);
    w.str("workflowInstanceKey"); w.integer(workflow_instance_key);
    w.str("activityInstanceKey"); w.integer(activity_instance_key);
    w.str("messageName"); w.str(message_name);
    w.str("correlationKey"); w.str(correlation_key);
    return w.b;
  }
};

// MessageRecord.java:26-42 (payload is a DocumentProperty: binary, {} by default; messageId "" by default)
struct MessageValue {
  bytes name;
  bytes correlation_key;
  int64_t ttl = 0;
  bytes payload = EMPTY_DOCUMENT;
  bytes message_id;
  bytes encode() const {
    MpWriter w;
    w.map_header(5);
    w.str("name"); w.str(name);
    w.str("correlationKey"); w.str(correlation_key);
    w.str("timeToLive"); w.integer(ttl);
    w.str("payload"); w.bin(payload);
    w.str("messageId"); w.str(message_id);
    return w.b;
  }
};

struct Record {
  int64_t position = 0;
  int64_t source_position = -1;
  int64_t key = -1;
  uint8_t record_type = RT_EVENT;
  uint8_t value_type = VT_WORKFLOW_INSTANCE;
  uint8_t intent = 0;
  uint8_t rejection_type = REJ_NULL;
  std::string rejection_reason;
  // log frame fields (LogStreamBatchWriterImpl.java:232-268, RecordMetadata.java:236-249 reset values)
  uint64_t request_id = UINT64_MAX;       // RecordMetadataEncoder.requestIdNullValue
  int32_t request_stream_id = INT32_MIN;  // RecordMetadataEncoder.requestStreamIdNullValue
  int32_t producer_id = -1;               // LogStreamBatchWriterImpl.reset :280 (client / external writers)
  uint8_t batch_flags = 0;                // DataFrameDescriptor BEGIN 0x80 / END 0x40 (ClaimedFragmentBatch.commit)
  WfValue wf;
  JobValue job;
  IncidentValue inc;
  WisValue wis;
  MsgSubValue msub;
  MessageValue msg;
  bytes raw_value;  // submitted from outside (zbref_submit_record): the log keeps the bytes as written
  bytes encode_value() const {
    if (!raw_value.empty()) return raw_value;
    switch (value_type) {
      case VT_WORKFLOW_INSTANCE: return wf.encode();
      case VT_JOB: return job.encode();
      case VT_INCIDENT: return inc.encode();
      case VT_WORKFLOW_INSTANCE_SUBSCRIPTION: return wis.encode();
      case VT_MESSAGE_SUBSCRIPTION: return msub.encode();
      case VT_MESSAGE: return msg.encode();
    }
    return bytes();
  }
};

// ------------------------------------------------------------------------------ executable model
enum ElemKind : uint8_t { K_PROCESS, K_START_EVENT, K_END_EVENT, K_SERVICE_TASK, K_SUB_PROCESS,
                          K_EXCLUSIVE_GATEWAY, K_INTERMEDIATE_CATCH, K_SEQUENCE_FLOW, K_PARALLEL_GATEWAY };

struct Element {
  ElemKind kind;
  bytes id;
  std::map<uint8_t, uint8_t> steps;  // intent -> BpmnStep (EnumMap)
  std::vector<Element*> outgoing;    // executable (walk) order
  std::vector<Element*> outgoing_with_condition;
  Element* default_flow = nullptr;
  Element* target = nullptr;         // sequence flow
  Element* start_event = nullptr;    // containers
  std::shared_ptr<CompiledCondition> condition;
  bytes job_type;
  int32_t retries = 3;
  bytes encoded_headers = EMPTY_DOCUMENT;  // JobRecord.NO_HEADERS
  bytes message_name;
  JsonPathQuery correlation_key;
  // zeebe:ioMapping (FlowNodeHandler.transformIoMappings, broker-core/.../transformation/handler/FlowNodeHandler.java:62-88)
  bool has_io_mapping = false;
  std::vector<Mapping> input_mappings, output_mappings;
  enum OutputBehavior : uint8_t { OB_UNSET = 0, OB_NONE, OB_MERGE, OB_OVERWRITE } output_behavior = OB_UNSET;
  int incoming = 0;                  // parallel gateway: sequence flows targeting it (join arity)
  uint8_t get_step(uint8_t intent) const {
    auto it = steps.find(intent);
    return it == steps.end() ? S_UNBOUND : it->second;
  }
};

struct Workflow {
  int64_t key;
  int32_t version;
  bytes bpmn_process_id;
  std::vector<std::unique_ptr<Element>> storage;
  std::unordered_map<bytes, Element*> by_id;
  Element* process = nullptr;
  bool has_parallel = false;
  Element* get(const bytes& id) const {
    auto it = by_id.find(id);
    return it == by_id.end() ? nullptr : it->second;
  }
};

// ------------------------------------------------------------------------------ transformer
// BpmnTransformer.java:52-83: two ModelWalker passes; each node's handlers run supertype-first
// (TypeHierarchyVisitor.java:34-41).
class Transformer {
 public:
  std::vector<std::unique_ptr<Workflow>> transform(const XmlNode& doc) {
    const XmlNode* defs = nullptr;
    for (auto& c : doc.children)
      if (c->name == "definitions") defs = c.get();
    if (!defs) throw ZbError("no definitions element");
    defs_ = defs;
    walk(defs, 1);
    walk(defs, 2);
    return std::move(workflows_);
  }

 private:
  const XmlNode* defs_ = nullptr;
  std::vector<std::unique_ptr<Workflow>> workflows_;
  Workflow* current_ = nullptr;
  uint8_t current_outgoing_step_ = S_NONE;

  static bool is_flow_node(const std::string& n) {
    return n == "startEvent" || n == "endEvent" || n == "serviceTask" || n == "subProcess" ||
           n == "exclusiveGateway" || n == "intermediateCatchEvent" || n == "parallelGateway" || n == "task" ||
           n == "userTask" || n == "receiveTask" || n == "sendTask" || n == "scriptTask" ||
           n == "businessRuleTask" || n == "manualTask" || n == "callActivity" || n == "inclusiveGateway" ||
           n == "eventBasedGateway" || n == "complexGateway" || n == "intermediateThrowEvent" ||
           n == "boundaryEvent" || n == "transaction";
  }
  static bool is_flow_element(const std::string& n) { return is_flow_node(n) || n == "sequenceFlow"; }
  static bool is_activity(const std::string& n) {
    return n == "serviceTask" || n == "subProcess" || n == "task" || n == "userTask" || n == "receiveTask" ||
           n == "sendTask" || n == "scriptTask" || n == "businessRuleTask" || n == "manualTask" ||
           n == "callActivity" || n == "transaction";
  }

  // ModelWalker.walk: children pushed with addFirst => siblings visited last-to-first
  void walk(const XmlNode* root, int pass) {
    std::deque<const XmlNode*> todo{root};
    while (!todo.empty()) {
      const XmlNode* n = todo.front();
      todo.pop_front();
      visit(n, pass);
      for (auto& c : n->children) todo.push_front(c.get());
    }
  }

  static std::vector<const XmlNode*> kids(const XmlNode* n, const char* name) {
    std::vector<const XmlNode*> out;
    for (auto& c : n->children)
      if (c->name == name) out.push_back(c.get());
    return out;
  }
  static const XmlNode* ext(const XmlNode* n, const char* name) {
    for (auto* e : kids(n, "extensionElements"))
      for (auto& c : e->children)
        if (c->name == name) return c.get();
    return nullptr;
  }
  static std::string id_of(const XmlNode* n) {
    const std::string* a = n->attr("id");
    return a ? *a : std::string();
  }

  void visit(const XmlNode* n, int pass) {
    const std::string& nm = n->name;
    if (pass == 1) {
      if (nm == "process") {  // CreateWorkflowHandler
        auto wf = std::make_unique<Workflow>();
        wf->bpmn_process_id = id_of(n);
        auto e = std::make_unique<Element>();
        e->kind = K_PROCESS;
        e->id = wf->bpmn_process_id;
        wf->process = e.get();
        wf->by_id[e->id] = e.get();
        wf->storage.push_back(std::move(e));
        current_ = wf.get();
        workflows_.push_back(std::move(wf));
      } else if (is_flow_element(nm)) {  // FlowElementHandler: ELEMENT_FACTORIES
        ElemKind k;
        if (nm == "endEvent") k = K_END_EVENT;
        else if (nm == "exclusiveGateway") k = K_EXCLUSIVE_GATEWAY;
        else if (nm == "intermediateCatchEvent") k = K_INTERMEDIATE_CATCH;
        else if (nm == "sequenceFlow") k = K_SEQUENCE_FLOW;
        else if (nm == "serviceTask") k = K_SERVICE_TASK;
        else if (nm == "startEvent") k = K_START_EVENT;
        else if (nm == "subProcess") k = K_SUB_PROCESS;
        else if (nm == "parallelGateway") k = K_PARALLEL_GATEWAY;  // EXTENSION (C4)
        else throw ZbError("unsupported element type: " + nm);  // factory lookup returns null (NPE)
        auto e = std::make_unique<Element>();
        e->kind = k;
        e->id = id_of(n);
        current_->by_id[e->id] = e.get();
        current_->storage.push_back(std::move(e));
      }
      return;
    }
    // pass 2
    if (nm == "process") {  // ProcessHandler
      for (auto& w : workflows_)
        if (w->bpmn_process_id == id_of(n)) current_ = w.get();
      Element* p = current_->process;
      p->steps[ELEMENT_READY] = S_APPLY_INPUT_MAPPING;
      p->steps[ELEMENT_ACTIVATED] = S_TRIGGER_START_EVENT;
      p->steps[ELEMENT_COMPLETING] = S_COMPLETE_PROCESS;
      p->steps[ELEMENT_TERMINATING] = S_TERMINATE_CONTAINED_INSTANCES;
      return;
    }
    if (!is_flow_element(nm)) return;
    Element* e = current_->get(id_of(n));
    if (nm == "sequenceFlow") {  // SequenceFlowHandler
      const std::vector<const XmlNode*> conds = kids(n, "conditionExpression");
      if (!conds.empty()) {
        auto c = std::make_shared<CompiledCondition>(create_condition(conds[0]->text));
        e->condition = c;
      }
      const std::string* sref = n->attr("sourceRef");
      const std::string* tref = n->attr("targetRef");
      Element* src = sref ? current_->get(*sref) : nullptr;
      Element* tgt = tref ? current_->get(*tref) : nullptr;
      if (!src || !tgt) throw ZbError("sequence flow with unknown source/target");
      src->outgoing.push_back(e);
      if (src->kind == K_EXCLUSIVE_GATEWAY && e->condition) src->outgoing_with_condition.push_back(e);
      e->target = tgt;
      uint8_t step;
      if (tgt->kind == K_SERVICE_TASK || tgt->kind == K_SUB_PROCESS || tgt->kind == K_INTERMEDIATE_CATCH)
        step = S_START_STATEFUL_ELEMENT;
      else if (tgt->kind == K_EXCLUSIVE_GATEWAY) step = S_ACTIVATE_GATEWAY;
      else if (tgt->kind == K_END_EVENT) step = S_TRIGGER_END_EVENT;
      else if (tgt->kind == K_PARALLEL_GATEWAY) {
        // EXTENSION: a flow into a join (>= 2 incoming flows) is an arrival, else it activates the gateway
        tgt->incoming = count_incoming(defs_, *tref);
        step = tgt->incoming >= 2 ? S_PARALLEL_MERGE : S_ACTIVATE_GATEWAY;
      }
      else throw ZbError("Unsupported element");
      e->steps[SEQUENCE_FLOW_TAKEN] = step;
      return;
    }
    // FlowNodeHandler (supertype first)
    {
      const XmlNode* io = ext(n, "ioMapping");
      if (io) {
        e->has_io_mapping = true;
        JsonPathCompiler jc;
        for (const XmlNode* m : kids(io, "input"))
          e->input_mappings.push_back({jc.compile(m->attr("source") ? *m->attr("source") : std::string()),
                                       m->attr("target") ? *m->attr("target") : std::string()});
        for (const XmlNode* m : kids(io, "output"))
          e->output_mappings.push_back({jc.compile(m->attr("source") ? *m->attr("source") : std::string()),
                                        m->attr("target") ? *m->attr("target") : std::string()});
        if (const std::string* b = io->attr("outputBehavior")) {
          if (*b == "none") e->output_behavior = Element::OB_NONE;
          else if (*b == "merge") e->output_behavior = Element::OB_MERGE;
          else if (*b == "overwrite") e->output_behavior = Element::OB_OVERWRITE;
          else throw ZbError("invalid outputBehavior: " + *b);
        }
      }
      size_t n_out = kids(n, "outgoing").size();  // FlowNode.getOutgoing(): <outgoing> references
      current_outgoing_step_ = n_out == 0 ? S_CONSUME_TOKEN : S_TAKE_SEQUENCE_FLOW;
    }
    if (is_activity(nm)) {  // ActivityHandler
      e->steps[ELEMENT_READY] = S_APPLY_INPUT_MAPPING;
      e->steps[ELEMENT_COMPLETING] = S_APPLY_OUTPUT_MAPPING;
      e->steps[ELEMENT_COMPLETED] = current_outgoing_step_;
      e->steps[ELEMENT_TERMINATED] = S_PROPAGATE_TERMINATION;
    }
    if (nm == "endEvent") {
      e->steps[END_EVENT_OCCURRED] = current_outgoing_step_;
    } else if (nm == "startEvent") {
      const XmlNode* scope = n->parent;
      if (scope->name == "subProcess") current_->get(id_of(scope))->start_event = e;
      else current_->process->start_event = e;
      e->steps[START_EVENT_OCCURRED] = current_outgoing_step_;
    } else if (nm == "exclusiveGateway") {
      const std::string* def = n->attr("default");
      if (def) e->default_flow = current_->get(*def);
      // bind: EXCLUSIVE_SPLIT iff the first *model-order* outgoing flow has a condition
      std::vector<const XmlNode*> outs = kids(n, "outgoing");
      bool first_has_cond = false;
      if (!outs.empty()) {
        std::string fid = outs[0]->text;
        // trim whitespace of the reference text
        while (!fid.empty() && (fid.back() == ' ' || fid.back() == '\n' || fid.back() == '\r' || fid.back() == '\t')) fid.pop_back();
        size_t b = 0;
        while (b < fid.size() && (fid[b] == ' ' || fid[b] == '\n' || fid[b] == '\r' || fid[b] == '\t')) b++;
        fid = fid.substr(b);
        const XmlNode* flow = find_by_id(defs_, fid);
        first_has_cond = flow && !kids(flow, "conditionExpression").empty();
      }
      e->steps[GATEWAY_ACTIVATED] = first_has_cond ? S_EXCLUSIVE_SPLIT : current_outgoing_step_;
    } else if (nm == "parallelGateway") {
      // EXTENSION: GATEWAY_ACTIVATED forks one token per outgoing flow (>= 1 required)
      if (kids(n, "outgoing").empty()) throw ZbError("parallel gateway without outgoing sequence flow");
      e->steps[GATEWAY_ACTIVATED] = S_PARALLEL_SPLIT;
      current_->has_parallel = true;
    } else if (nm == "serviceTask") {
      const XmlNode* td = ext(n, "taskDefinition");
      if (td) {
        if (const std::string* t = td->attr("type")) e->job_type = *t;
        if (const std::string* r = td->attr("retries")) e->retries = std::stoi(*r);
      }
      const XmlNode* th = ext(n, "taskHeaders");
      if (th) {
        std::vector<const XmlNode*> hs = kids(th, "header");
        if (hs.empty()) e->encoded_headers = bytes();  // UnsafeBuffer(0,0)
        else {
          MpWriter w;
          w.map_header((uint32_t)hs.size());
          for (auto* h : hs) {
            w.str(h->attr("key") ? *h->attr("key") : std::string());
            w.str(h->attr("value") ? *h->attr("value") : std::string());
          }
          e->encoded_headers = w.b;
        }
      }
      e->steps[ELEMENT_ACTIVATED] = S_CREATE_JOB;
      e->steps[ELEMENT_TERMINATING] = S_TERMINATE_JOB_TASK;
    } else if (nm == "subProcess") {
      e->steps[ELEMENT_ACTIVATED] = S_TRIGGER_START_EVENT;
      e->steps[ELEMENT_TERMINATING] = S_TERMINATE_CONTAINED_INSTANCES;
    } else if (nm == "intermediateCatchEvent") {
      std::vector<const XmlNode*> defsv = kids(n, "messageEventDefinition");
      if (defsv.empty()) throw ZbError("intermediate catch event without message");
      const std::string* mref = defsv[0]->attr("messageRef");
      const XmlNode* msg = mref ? find_by_id(defs_, *mref) : nullptr;
      if (!msg) throw ZbError("message not found");
      const XmlNode* sub = ext(msg, "subscription");
      JsonPathCompiler jc;
      e->correlation_key = jc.compile(sub && sub->attr("correlationKey") ? *sub->attr("correlationKey") : "");
      e->message_name = msg->attr("name") ? *msg->attr("name") : std::string();
      e->steps[ELEMENT_READY] = S_APPLY_INPUT_MAPPING;
      e->steps[ELEMENT_ACTIVATED] = S_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE;
      e->steps[ELEMENT_COMPLETING] = S_APPLY_OUTPUT_MAPPING;
      e->steps[ELEMENT_COMPLETED] = current_outgoing_step_;
      e->steps[ELEMENT_TERMINATING] = S_TERMINATE_ELEMENT;
      e->steps[ELEMENT_TERMINATED] = S_PROPAGATE_TERMINATION;
    }
  }

  static int count_incoming(const XmlNode* n, const std::string& id) {
    int c = 0;
    if (n->name == "sequenceFlow") {
      const std::string* t = n->attr("targetRef");
      if (t && *t == id) c++;
    }
    for (auto& k : n->children) c += count_incoming(k.get(), id);
    return c;
  }

  static const XmlNode* find_by_id(const XmlNode* n, const std::string& id) {
    const std::string* a = n->attr("id");
    if (a && *a == id) return n;
    for (auto& c : n->children)
      if (const XmlNode* f = find_by_id(c.get(), id)) return f;
    return nullptr;
  }
};

// ------------------------------------------------------------------------------ index
struct ElementInstance {  // ElementInstance.java:30-111
  int64_t key;
  ElementInstance* parent;
  uint8_t state;
  WfValue value;
  std::vector<ElementInstance*> children;
  int64_t job_key = 0;
  // EXTENSION (C4): live tokens of a scope and arrivals per parallel join
  int32_t tokens = 0;
  std::map<const void*, int32_t> joins;
};

struct ElementInstanceIndex {  // ElementInstanceIndex.java:25-65
  std::unordered_map<int64_t, std::unique_ptr<ElementInstance>> instances;
  ElementInstance* new_instance(ElementInstance* parent, int64_t key, const WfValue& v, uint8_t state) {
    auto ei = std::make_unique<ElementInstance>();
    ei->key = key;
    ei->parent = parent;
    if (parent) parent->children.push_back(ei.get());
    ei->state = state;
    ei->value = v;
    ElementInstance* raw = ei.get();
    auto it = instances.find(key);
    if (it != instances.end()) graveyard.push_back(std::move(it->second));  // replaced object stays referenced
    instances[key] = std::move(ei);
    return raw;
  }
  ElementInstance* get(int64_t key) {
    auto it = instances.find(key);
    return it == instances.end() ? nullptr : it->second.get();
  }
  void remove(int64_t key) {
    auto it = instances.find(key);
    if (it == instances.end()) return;
    ElementInstance* ei = it->second.get();
    if (ei->parent) {
      auto& ch = ei->parent->children;
      for (size_t i = 0; i < ch.size(); i++)
        if (ch[i] == ei) { ch.erase(ch.begin() + i); break; }
    }
    graveyard.push_back(std::move(it->second));  // children may still point at it
    instances.erase(it);
  }
  std::vector<std::unique_ptr<ElementInstance>> graveyard;
};

struct KeyGenerator {  // KeyGenerator.java:28-56
  int64_t next;
  int64_t step;
  int64_t next_key() { int64_t k = next; next += step; return k; }
};

// A side effect the processors hand to the subscription transport (SubscriptionCommandSender.java:83-128)
struct SideEffect {
  int kind;                 // 1 = open message subscription, 2 = correlate workflow instance subscription
  int64_t workflow_instance_key;
  int64_t activity_instance_key;
  bytes message_name;
  bytes correlation_key;    // kind 1
  int32_t partition;        // target: kind 1 abs(hash % P) (SubscriptionCommandSender.java:105-109), kind 2 the
                            // workflow instance partition (:111-128)
  int32_t wf_partition;     // kind 1: the sending (workflow) partition
  bytes payload;            // kind 2: the message payload
};

// ------------------------------------------------------------------------------ engine
class Engine {
 public:
  int partition_id = 0;
  int partition_count = 1;
  std::vector<Record> log;
  std::vector<SideEffect> side_effects;
  KeyGenerator wf_keys{1, 5};
  KeyGenerator job_keys{2, 5};
  KeyGenerator msg_keys{0, 1};  // message stream processor (MessageService.java:91)
  // MessageSubscriptionDataStore / MessageDataStore: insertion-ordered lists, linear scans
  struct StoredSub { int32_t wfp; int64_t wik, aik; bytes name, ck; };
  struct StoredMsg { bytes name, ck, payload, id; int64_t ttl, key, deadline; };  // MessageDataStore.Message
  int64_t clock_ms = 0;  // ActorClock.currentTimeMillis() of the processing (MessageDataStore.Message deadline)
  std::vector<StoredSub> subs;
  std::vector<StoredMsg> msgs;
  ElementInstanceIndex index;
  std::vector<std::unique_ptr<Workflow>> workflows;
  std::map<std::pair<int64_t, bytes>, bytes> job_payloads;  // (workflow key, activity id) -> completion payload
  int64_t created = 0, completed = 0, canceled = 0;
  int64_t transitions = 0;  // WORKFLOW_INSTANCE events written (streamprocessor_events_count{written}, WF)
  size_t processed = 0;
  // canonical job harness on; off: JOB CREATE commands wait for job events submitted
  // from outside (the job stream processor's JOB CREATED / JOB COMPLETED records, zbref_submit_record)
  bool harness = true;
  // the job stream processor (JobInstanceStreamProcessor.java:70-242) on the same log, as a FIFO participant:
  // JOB commands are processed at their log position; job states by key (JobStateController)
  bool job_processor = false;
  enum JobState : uint8_t { JS_NONE = 0, JS_CREATED, JS_ACTIVATED, JS_FAILED, JS_TIMED_OUT };
  std::unordered_map<int64_t, uint8_t> job_states;
  std::string last_error;

  // ZeebeIoMappingValidator (broker-core/.../validation/ZeebeIoMappingValidator.java:36-57), the model's
  // ZeebeIoMappingValidator (bpmn-model/.../validation/zeebe/ZeebeIoMappingValidator.java:31-39) and
  // ZeebeExpressionValidator.validateJsonPath (:42-54) for every source and target
  static void validate_io_mapping(const Element& e) {
    auto root_target = [](const std::vector<Mapping>& ms) {
      for (auto& m : ms)
        if (m.target == "$") return true;
      return false;
    };
    if (e.input_mappings.size() > 1 && root_target(e.input_mappings))
      throw ZbError("Invalid inputs: When using $ as target, no other input can be defined");
    if (e.output_mappings.size() > 1 && root_target(e.output_mappings))
      throw ZbError("Invalid outputs: When using $ as target, no other output can be defined");
    if (e.output_behavior == Element::OB_NONE && !e.output_mappings.empty())
      throw ZbError("Output behavior 'none' cannot be used in combination without zeebe:output elements");
    JsonPathCompiler jc;
    for (const auto* ms : {&e.input_mappings, &e.output_mappings})
      for (auto& m : *ms) {
        for (const bytes& path : {m.source.expression, m.target}) {
          JsonPathQuery q = jc.compile(path);
          if (!q.valid()) throw ZbError("JSON path query is invalid: " + q.error);
          // PROHIBITED_PATHS_REGEX "(\\.\\*)|(\\[.*,.*\\])"
          if (path.find(".*") != std::string::npos) throw ZbError("This JSON path query is not supported");
          const size_t lb = path.find('[');
          if (lb != std::string::npos) {
            const size_t comma = path.find(',', lb + 1);
            if (comma != std::string::npos && path.find(']', comma + 1) != std::string::npos)
              throw ZbError("This JSON path query is not supported");
          }
        }
      }
  }

  void deploy(const std::string& xml, int64_t key, int32_t version) {
    XmlReader xr;
    auto doc = xr.parse(xml);
    Transformer tr;
    auto wfs = tr.transform(*doc);
    int64_t k = key;
    for (auto& w : wfs) {
      for (auto& e : w->storage) {
        if (e->has_io_mapping) validate_io_mapping(*e);
        if (e->condition && !e->condition->valid) throw ZbError("invalid condition: " + e->condition->error);
      }
      w->key = k++;
      w->version = version;
      workflows.push_back(std::move(w));
    }
  }

  Workflow* by_key(int64_t key) {
    for (auto& w : workflows)
      if (w->key == key) return w.get();
    return nullptr;
  }
  Workflow* by_id_version(const bytes& id, int32_t v) {
    for (auto& w : workflows)
      if (w->bpmn_process_id == id && w->version == v) return w.get();
    return nullptr;
  }
  Workflow* latest(const bytes& id) {
    Workflow* best = nullptr;
    for (auto& w : workflows)
      if (w->bpmn_process_id == id && (!best || w->version > best->version)) best = w.get();
    return best;
  }

  int64_t pos_base = 0;  // the position of log[0] (zbref_set_position_base; the engine's zb_log_start)

  void append(Record r) {
    r.position = pos_base + (int64_t)log.size();
    log.push_back(std::move(r));
  }

  void submit_create(const bytes& process_id, int32_t version, int64_t workflow_key, const bytes& payload) {
    Record r;
    r.record_type = RT_COMMAND;
    r.value_type = VT_WORKFLOW_INSTANCE;
    r.intent = CREATE;
    r.key = -1;
    r.wf.bpmn_process_id = process_id;
    r.wf.version = version;
    r.wf.workflow_key = workflow_key;
    r.wf.set_payload(payload);
    append(std::move(r));
  }
  void submit_cancel(int64_t key) {
    Record r;
    r.record_type = RT_COMMAND;
    r.intent = CANCEL;
    r.key = key;
    append(std::move(r));
  }
  void submit_correlate(int64_t wf_instance_key, int64_t activity_instance_key, const bytes& name,
                        const bytes& payload) {
    Record r;
    r.record_type = RT_COMMAND;
    r.value_type = VT_WORKFLOW_INSTANCE_SUBSCRIPTION;
    r.intent = WIS_CORRELATE;
    r.key = pos_base + (int64_t)log.size();  // positionAsKey (SubscriptionApiCommandMessageHandler.java:131-151)
    r.wis.workflow_instance_key = wf_instance_key;
    r.wis.activity_instance_key = activity_instance_key;
    r.wis.message_name = name;
    r.wis.payload = payload.empty() ? EMPTY_DOCUMENT : payload;
    append(std::move(r));
  }

  // A record written to the partition log by another writer (client API, job stream processor,
  // subscription API), given as its reference msgpack value: UnpackedObject.wrap reads the declared
  // properties (ObjectValue.java:93-131); the log keeps the bytes as written.
  void submit_record(uint8_t record_type, uint8_t value_type, uint8_t intent, int64_t key, const bytes& value) {
    Record r;
    r.record_type = record_type;
    r.value_type = value_type;
    r.intent = intent;
    r.key = key;
    r.raw_value = value;
    if (value_type == VT_WORKFLOW_INSTANCE) decode_wf(value, r.wf);
    else if (value_type == VT_JOB) decode_job(value, r.job);
    else if (value_type == VT_WORKFLOW_INSTANCE_SUBSCRIPTION) decode_wis(value, r.wis);
    else if (value_type == VT_MESSAGE) decode_msg(value, r.msg);
    else throw ZbError("unsupported value type for submit");
    if (value.empty()) r.raw_value.clear();
    // a MESSAGE DELETE command is written by the time-to-live checker's own command writer (producer id 0)
    if (record_type == RT_COMMAND && value_type == VT_MESSAGE && intent == MSG_DELETE) r.producer_id = 0;
    if (record_type == RT_COMMAND && value_type == VT_WORKFLOW_INSTANCE_SUBSCRIPTION && intent == WIS_CORRELATE)
      r.key = pos_base + (int64_t)log.size();  // positionAsKey (SubscriptionApiCommandMessageHandler.java:131-151)
    append(std::move(r));
  }

  static bytes read_str(MpReader& rd) {
    uint32_t n = rd.read_string_length();
    if (rd.off + n > rd.cap) throw ZbError("Index out of bounds");
    bytes b((const char*)rd.buf + rd.off, n);
    rd.off += n;
    return b;
  }
  static bytes read_doc(MpReader& rd) {  // DocumentProperty: msgpack binary, nil / empty -> {}
    uint32_t n = rd.read_binary_length();
    if (rd.off + n > rd.cap) throw ZbError("Index out of bounds");
    bytes b((const char*)rd.buf + rd.off, n);
    rd.off += n;
    if (b.empty() || (b.size() == 1 && (uint8_t)b[0] == 0xc0)) return EMPTY_DOCUMENT;
    return b;
  }
  template <class F>
  static void for_props(MpReader& rd, F f) {
    uint32_t n = rd.read_map_header();
    for (uint32_t i = 0; i < n; i++) {
      bytes k = read_str(rd);
      if (!f(k, rd)) rd.skip_values(1);
    }
  }
  static void decode_wf(const bytes& b, WfValue& v) {  // WorkflowInstanceRecord.java:39-60
    if (b.empty()) return;
    MpReader rd(b);
    for_props(rd, [&](const bytes& k, MpReader& r) {
      if (k == "bpmnProcessId") v.bpmn_process_id = read_str(r);
      else if (k == "version") v.version = (int32_t)r.read_integer();
      else if (k == "workflowKey") v.workflow_key = r.read_integer();
      else if (k == "workflowInstanceKey") v.workflow_instance_key = r.read_integer();
      else if (k == "activityId") v.activity_id = read_str(r);
      else if (k == "payload") v.payload = read_doc(r);
      else if (k == "scopeInstanceKey") v.scope_instance_key = r.read_integer();
      else return false;
      return true;
    });
  }
  static void decode_job(const bytes& b, JobValue& v) {  // JobRecord.java:35-53, JobHeaders.java:33-51
    if (b.empty()) return;
    MpReader rd(b);
    for_props(rd, [&](const bytes& k, MpReader& r) {
      if (k == "deadline") v.deadline = r.read_integer();
      else if (k == "worker") v.worker = read_str(r);
      else if (k == "retries") v.retries = (int32_t)r.read_integer();
      else if (k == "type") v.type = read_str(r);
      else if (k == "headers") {
        for_props(r, [&](const bytes& hk, MpReader& hr) {
          if (hk == "bpmnProcessId") v.h_bpmn_process_id = read_str(hr);
          else if (hk == "workflowDefinitionVersion") v.h_version = (int32_t)hr.read_integer();
          else if (hk == "workflowKey") v.h_workflow_key = hr.read_integer();
          else if (hk == "workflowInstanceKey") v.h_workflow_instance_key = hr.read_integer();
          else if (hk == "activityId") v.h_activity_id = read_str(hr);
          else if (hk == "activityInstanceKey") v.h_activity_instance_key = hr.read_integer();
          else return false;
          return true;
        });
      } else if (k == "customHeaders") {
        size_t st = r.off;
        r.skip_values(1);
        v.custom_headers = bytes((const char*)r.buf + st, r.off - st);
      } else if (k == "payload") v.payload = read_doc(r);
      else return false;
      return true;
    });
  }
  static void decode_msg(const bytes& b, MessageValue& v) {  // MessageRecord.java:26-42
    if (b.empty()) return;
    MpReader rd(b);
    for_props(rd, [&](const bytes& k, MpReader& r) {
      if (k == "name") v.name = read_str(r);
      else if (k == "correlationKey") v.correlation_key = read_str(r);
      else if (k == "timeToLive") v.ttl = r.read_integer();
      else if (k == "payload") v.payload = read_doc(r);
      else if (k == "messageId") v.message_id = read_str(r);
      else return false;
      return true;
    });
  }
  // MessageTimeToLiveChecker.run :44-68 at `now`: a DELETE command (key = message key, the stored message's
  // name / correlation key / ttl / payload / id) for every stored message whose deadline has passed, in store
  // order, written by the checker's own command writer (no source event position, producer id 0)
  size_t check_ttl(int64_t now) {
    size_t n = 0;
    for (const StoredMsg& m : msgs) {
      if (m.deadline > now) continue;
      Record r;
      r.record_type = RT_COMMAND;
      r.value_type = VT_MESSAGE;
      r.intent = MSG_DELETE;
      r.key = m.key;
      r.msg.name = m.name;
      r.msg.correlation_key = m.ck;
      r.msg.ttl = m.ttl;
      r.msg.payload = m.payload;
      r.msg.message_id = m.id;
      r.producer_id = 0;
      append(std::move(r));
      n++;
    }
    return n;
  }
  static void decode_wis(const bytes& b, WisValue& v) {  // WorkflowInstanceSubscriptionRecord.java:26-38
    if (b.empty()) return;
    MpReader rd(b);
    for_props(rd, [&](const bytes& k, MpReader& r) {
      if (k == "workflowInstanceKey") v.workflow_instance_key = r.read_integer();
      else if (k == "activityInstanceKey") v.activity_instance_key = r.read_integer();
      else if (k == "messageName") v.message_name = read_str(r);
      else if (k == "payload") v.payload = read_doc(r);
      else return false;
      return true;
    });
  }

  // SubscriptionApiCommandMessageHandler.onOpenMessageSubscription :94-110 (command key = position)
  void submit_open(int32_t wfp, int64_t wik, int64_t aik, const bytes& name, const bytes& ck) {
    Record r;
    r.record_type = RT_COMMAND;
    r.value_type = VT_MESSAGE_SUBSCRIPTION;
    r.intent = MSUB_OPEN;
    r.key = pos_base + (int64_t)log.size();
    r.msub.wf_partition = wfp;
    r.msub.workflow_instance_key = wik;
    r.msub.activity_instance_key = aik;
    r.msub.message_name = name;
    r.msub.correlation_key = ck;
    append(std::move(r));
  }
  // ClientApiMessageHandler.handleExecuteCommandRequest :90-162: MESSAGE PUBLISH command, null key
  void submit_publish(const bytes& name, const bytes& ck, int64_t ttl, const bytes& payload, const bytes& id) {
    Record r;
    r.record_type = RT_COMMAND;
    r.value_type = VT_MESSAGE;
    r.intent = MSG_PUBLISH;
    r.key = -1;
    r.msg.name = name;
    r.msg.correlation_key = ck;
    r.msg.ttl = ttl;
    r.msg.payload = (payload.empty() || (payload.size() == 1 && (uint8_t)payload[0] == 0xc0)) ? EMPTY_DOCUMENT : payload;
    r.msg.message_id = id;
    append(std::move(r));
  }

  size_t run(size_t max_records = SIZE_MAX) {
    size_t n = 0;
    while (processed < log.size() && n < max_records) {
      process(processed);
      processed++;
      n++;
    }
    return n;
  }

  // ---- typed writer (TypedStreamWriterImpl / TypedCommandWriterImpl) for one processed record
  struct Writer {
    Engine* eng;
    bool batch = false;
    std::vector<Record> staged;
    void stage(Record r) {
      if (batch) staged.push_back(std::move(r));
      else { staged.clear(); staged.push_back(std::move(r)); }
    }
    void new_batch() { batch = true; staged.clear(); }
  };

 private:
  Writer* w_ = nullptr;
  ElInterpreter interp_;
  JsonPathExecutor jp_;

  // ElementInstanceWriter.writeNewEvent :64-84
  int64_t write_new_wf_event(uint8_t intent, const WfValue& v) {
    int64_t key = wf_keys.next_key();
    Record r;
    r.key = key; r.record_type = RT_EVENT; r.value_type = VT_WORKFLOW_INSTANCE; r.intent = intent; r.wf = v;
    w_->stage(std::move(r));
    if (intent == ELEMENT_READY) {
      if (v.scope_instance_key >= 0) index.new_instance(index.get(v.scope_instance_key), key, v, intent);
      else index.new_instance(nullptr, key, v, intent);
    }
    return key;
  }
  // ElementInstanceWriter.writeFollowUpEvent :86-110
  void write_followup_wf_event(int64_t key, uint8_t intent, const WfValue& v) {
    Record r;
    r.key = key; r.record_type = RT_EVENT; r.value_type = VT_WORKFLOW_INSTANCE; r.intent = intent; r.wf = v;
    w_->stage(std::move(r));
    if (intent == ELEMENT_COMPLETED || intent == ELEMENT_TERMINATED) {
      index.remove(key);
    } else {
      ElementInstance* ei = index.get(key);
      if (!ei) throw ZbError("NullPointerException: no element instance for follow-up event");
      ei->state = intent;
      ei->value = v;
    }
    if (key == v.workflow_instance_key) {
      if (intent == ELEMENT_TERMINATED) canceled++;
      else if (intent == ELEMENT_COMPLETED) completed++;
    }
  }
  // plain TypedStreamWriter.writeFollowUpEvent (no index side effects)
  void stage_event(int64_t key, uint8_t vt, uint8_t intent, const Record& proto) {
    Record r = proto;
    r.key = key; r.record_type = RT_EVENT; r.value_type = vt; r.intent = intent;
    w_->stage(std::move(r));
  }
  void write_rejection(const Record& cmd, uint8_t type, const std::string& reason) {
    Record r = cmd;
    r.record_type = RT_REJECTION;
    r.rejection_type = type;
    r.rejection_reason = reason;
    w_->stage(std::move(r));
  }

  // BpmnStepContext.raiseIncident :141-162
  void raise_incident(const Record& rec, uint8_t error_type, const std::string& msg) {
    Record r;
    r.key = -1; r.record_type = RT_COMMAND; r.value_type = VT_INCIDENT; r.intent = INCIDENT_CREATE;
    r.inc.error_type = error_type;
    r.inc.error_message = msg;
    r.inc.failure_event_position = rec.position;
    r.inc.activity_instance_key = rec.key;
    r.inc.bpmn_process_id = rec.wf.bpmn_process_id;
    r.inc.workflow_instance_key = rec.wf.workflow_instance_key;
    r.inc.activity_id = rec.wf.activity_id;
    w_->stage(std::move(r));
  }

  void process(size_t pos) {
    const Record rec = log[pos];  // copy: the log grows while processing
    Writer w{this};
    w_ = &w;
    try {
      dispatch(rec);
    } catch (const ZbError& e) {
      // StreamProcessorController.onFailure: the partition stops processing
      last_error = std::string("processing failed at position ") + std::to_string(pos_base + (int64_t)pos) + ": " + e.what();
      throw;
    }
    w_ = nullptr;
    // TypedStreamProcessor: writer.configureSourceContext(streamProcessorId, position) (StreamProcessorIds.java:23-39):
    // the job processor (harness) 10, the message processor 90, the workflow instance processor 70
    const int32_t producer = rec.value_type == VT_JOB && rec.record_type == RT_COMMAND ? 10
                           : (rec.value_type == VT_MESSAGE || rec.value_type == VT_MESSAGE_SUBSCRIPTION) ? 90 : 70;
    const size_t nst = w.staged.size();
    for (size_t k = 0; k < nst; k++) {
      Record& r = w.staged[k];
      r.raw_value.clear();  // follow-ups are encoded from their value objects
      if (r.value_type == VT_WORKFLOW_INSTANCE && r.record_type == RT_EVENT) transitions++;
      r.source_position = rec.position;
      r.producer_id = producer;
      // ClaimedFragmentBatch.commit :130-147: batch flags only when the batch holds more than one fragment
      r.batch_flags = nst > 1 ? (k == 0 ? 0x80 : (k + 1 == nst ? 0x40 : 0)) : 0;
      // RecordMetadata.reset on every write; only the CREATE processor copies the command's request
      // metadata, onto CREATED and onto its rejection (WorkflowInstanceStreamProcessor.java:254-257, :370-377)
      const bool keeps = r.value_type == VT_WORKFLOW_INSTANCE &&
                         ((r.record_type == RT_EVENT && r.intent == CREATED) ||
                          (r.record_type == RT_REJECTION && r.intent == CREATE));
      r.request_id = keeps ? rec.request_id : UINT64_MAX;
      r.request_stream_id = keeps ? rec.request_stream_id : INT32_MIN;
      append(std::move(r));
    }
  }

  void dispatch(const Record& rec) {
    if (rec.value_type == VT_WORKFLOW_INSTANCE) {
      if (rec.record_type == RT_COMMAND) {
        if (rec.intent == CREATE) process_create(rec);
        else if (rec.intent == CANCEL) process_cancel(rec);
        else if (rec.intent == UPDATE_PAYLOAD) process_update_payload(rec);
      } else if (rec.record_type == RT_EVENT) {
        switch (rec.intent) {
          case CREATED:  // WorkflowInstanceCreatedEventProcessor :380-394
            created++;
            index.new_instance(nullptr, rec.key, rec.wf, ELEMENT_READY);
            break;
          case SEQUENCE_FLOW_TAKEN: case ELEMENT_READY: case ELEMENT_ACTIVATED: case ELEMENT_COMPLETING:
          case START_EVENT_OCCURRED: case END_EVENT_OCCURRED: case GATEWAY_ACTIVATED: case ELEMENT_COMPLETED:
          case ELEMENT_TERMINATING: case ELEMENT_TERMINATED:
            bpmn_step(rec);
            break;
          default: break;
        }
      }
    } else if (rec.value_type == VT_JOB) {
      if (rec.record_type == RT_COMMAND && job_processor) process_job_command(rec);
      else if (rec.record_type == RT_COMMAND && rec.intent == JOB_CREATE) { if (harness) harness_job_create(rec); }
      else if (rec.record_type == RT_EVENT && rec.intent == JOB_CREATED) process_job_created(rec);
      else if (rec.record_type == RT_EVENT && rec.intent == JOB_COMPLETED) process_job_completed(rec);
    } else if (rec.value_type == VT_WORKFLOW_INSTANCE_SUBSCRIPTION) {
      if (rec.record_type == RT_COMMAND && rec.intent == WIS_CORRELATE) process_correlate(rec);
    } else if (rec.value_type == VT_MESSAGE_SUBSCRIPTION) {  // message stream processor (MessageService.java:90-129)
      if (rec.record_type == RT_COMMAND && rec.intent == MSUB_OPEN) process_open_subscription(rec);
    } else if (rec.value_type == VT_MESSAGE) {
      if (rec.record_type == RT_COMMAND && rec.intent == MSG_PUBLISH) process_publish(rec);
      else if (rec.record_type == RT_COMMAND && rec.intent == MSG_DELETE) process_delete_message(rec);
    }
  }

  // CreateWorkflowInstanceEventProcessor :224-368 (all workflows are deployed locally; a miss
  // rejects with BAD_VALUE "Workflow is not deployed" as after a failed fetch)
  void process_create(const Record& cmd) {
    Record c = cmd;
    int64_t instance_key = wf_keys.next_key();
    c.wf.workflow_instance_key = instance_key;
    Workflow* wf = nullptr;
    if (c.wf.workflow_key <= 0) {
      if (c.wf.version > 0) {
        wf = by_id_version(c.wf.bpmn_process_id, c.wf.version);
        if (wf) c.wf.workflow_key = wf->key;
      } else {
        wf = latest(c.wf.bpmn_process_id);
        if (wf) { c.wf.workflow_key = wf->key; c.wf.version = wf->version; }
      }
    } else {
      wf = by_key(c.wf.workflow_key);
      if (wf) { c.wf.version = wf->version; c.wf.bpmn_process_id = wf->bpmn_process_id; }
    }
    if (!wf) {
      write_rejection(c, REJ_BAD_VALUE, "Workflow is not deployed");
      return;
    }
    c.wf.activity_id = c.wf.bpmn_process_id;
    w_->new_batch();
    Record a; a.key = instance_key; a.record_type = RT_EVENT; a.value_type = VT_WORKFLOW_INSTANCE;
    a.intent = CREATED; a.wf = c.wf;
    w_->stage(a);
    a.intent = ELEMENT_READY;
    w_->stage(a);
  }

  void process_cancel(const Record& cmd) {  // CancelWorkflowInstanceProcessor :511-555
    ElementInstance* wi = index.get(cmd.key);
    bool can = wi && (wi->state == ELEMENT_READY || wi->state == ELEMENT_ACTIVATED || wi->state == ELEMENT_COMPLETING);
    if (!can) {
      write_rejection(cmd, REJ_NOT_APPLICABLE, "Workflow instance is not running");
      return;
    }
    // workflowInstance.getValue() is the live indexed object (ElementInstance.java:67-69): setPayload
    // mutates the index too, so the instance's later TERMINATED (PropagateTerminationHandler :29-40)
    // carries the emptied payload.
    wi->value.payload = EMPTY_DOCUMENT;
    WfValue v = wi->value;
    w_->new_batch();
    Record a; a.key = cmd.key; a.record_type = RT_EVENT; a.value_type = VT_WORKFLOW_INSTANCE; a.wf = v;
    a.intent = CANCELING; w_->stage(a);
    a.intent = ELEMENT_TERMINATING; w_->stage(a);
    wi->state = ELEMENT_TERMINATING;
  }

  void process_update_payload(const Record& cmd) {  // UpdatePayloadProcessor :557-576
    ElementInstance* wi = index.get(cmd.wf.workflow_instance_key);
    if (wi) {
      wi->value.set_payload(cmd.wf.payload);
      Record a = cmd; a.record_type = RT_EVENT; a.intent = PAYLOAD_UPDATED;
      if (a.key < 0) a.key = wf_keys.next_key();  // CommandProcessorImpl.accept :77-84: null key -> new key
      w_->stage(a);
    } else {
      write_rejection(cmd, REJ_NOT_APPLICABLE, "Workflow instance is not running");
    }
  }

  void process_job_created(const Record& rec) {  // JobCreatedProcessor :408-426
    int64_t aik = rec.job.h_activity_instance_key;
    if (aik > 0) {
      ElementInstance* ai = index.get(aik);
      if (ai) ai->job_key = rec.key;
    }
  }
  void process_job_completed(const Record& rec) {  // JobCompletedEventProcessor :428-453
    int64_t aik = rec.job.h_activity_instance_key;
    ElementInstance* ai = index.get(aik);
    if (ai) {
      WfValue v = ai->value;
      v.set_payload(rec.job.payload);
      Record a; a.key = aik; a.record_type = RT_EVENT; a.value_type = VT_WORKFLOW_INSTANCE;
      a.intent = ELEMENT_COMPLETING; a.wf = v;
      w_->stage(a);
      ai->state = ELEMENT_COMPLETING;
      ai->job_key = -1;
      ai->value = v;
    }
  }
  void process_correlate(const Record& rec) {  // CorrelateWorkflowInstanceSubscription :455-509
    ElementInstance* ei = index.get(rec.wis.activity_instance_key);
    if (!ei) {
      write_rejection(rec, REJ_NOT_APPLICABLE, "activity is not active anymore");
      return;
    }
    WfValue v = ei->value;
    v.set_payload(rec.wis.payload);
    w_->new_batch();
    Record a = rec; a.record_type = RT_EVENT; a.intent = WIS_CORRELATED;
    w_->stage(a);
    Record b; b.key = rec.wis.activity_instance_key; b.record_type = RT_EVENT; b.value_type = VT_WORKFLOW_INSTANCE;
    b.intent = ELEMENT_COMPLETING; b.wf = v;
    w_->stage(b);
    ei->state = ELEMENT_COMPLETING;
    ei->value = v;
  }

  // OpenMessageSubscriptionProcessor.processRecord :56-83
  void process_open_subscription(const Record& rec) {
    const MsgSubValue& v = rec.msub;
    for (const StoredMsg& m : msgs) {  // MessageDataStore.findMessage: first match in insertion order
      if (m.name == v.message_name && m.ck == v.correlation_key) {
        side_effects.push_back({2, v.workflow_instance_key, v.activity_instance_key, v.message_name, bytes(),
                                v.wf_partition, v.wf_partition, m.payload});
        break;
      }
    }
    stage_event(rec.key, VT_MESSAGE_SUBSCRIPTION, MSUB_OPENED, rec);
    subs.push_back({v.wf_partition, v.workflow_instance_key, v.activity_instance_key, v.message_name,
                    v.correlation_key});
  }
  // PublishMessageProcessor.processRecord :58-105 + correlateMessage :107-124
  void process_publish(const Record& rec) {
    const MessageValue& v = rec.msg;
    if (!v.message_id.empty()) {  // MessageDataStore.hasMessage
      for (const StoredMsg& m : msgs) {
        if (!m.id.empty() && m.id == v.message_id && m.name == v.name && m.ck == v.correlation_key) {
          write_rejection(rec, REJ_BAD_VALUE, "message with id '" + v.message_id + "' is already published");
          return;
        }
      }
    }
    w_->new_batch();
    const int64_t key = msg_keys.next_key();
    Record a = rec;
    a.key = key; a.record_type = RT_EVENT; a.intent = MSG_PUBLISHED;
    w_->stage(a);
    for (const StoredSub& sb : subs)  // MessageSubscriptionDataStore.findSubscriptions (insertion order)
      if (sb.name == v.name && sb.ck == v.correlation_key)
        side_effects.push_back({2, sb.wik, sb.aik, v.name, bytes(), sb.wfp, sb.wfp, v.payload});
    if (v.ttl > 0) {
      msgs.push_back({v.name, v.correlation_key, v.payload, v.message_id, v.ttl, key, v.ttl + clock_ms});
    } else {
      Record d = rec;
      d.key = key; d.record_type = RT_EVENT; d.intent = MSG_DELETED;
      w_->stage(d);
    }
  }
  // DeleteMessageProcessor.processRecord :36-45
  void process_delete_message(const Record& rec) {
    stage_event(rec.key, VT_MESSAGE, MSG_DELETED, rec);
    for (size_t i = 0; i < msgs.size(); i++)
      if (msgs[i].key == rec.key) { msgs.erase(msgs.begin() + i); break; }
  }

  // JobInstanceStreamProcessor :98-242. CommandProcessorImpl: accept -> writeFollowUpEvent(key, intent, command
  // value) with a new key for a null command key (:73-82); reject -> writeRejection(command, type, reason)
  void process_job_command(const Record& cmd) {
    auto st = [&]() -> uint8_t {
      auto it = job_states.find(cmd.key);
      return it == job_states.end() ? JS_NONE : it->second;
    };
    auto accept = [&](uint8_t intent, int64_t key) {
      Record a = cmd;
      a.key = key; a.record_type = RT_EVENT; a.intent = intent;
      w_->stage(std::move(a));
    };
    const uint8_t s0 = st();
    switch (cmd.intent) {
      case JOB_CREATE: {  // CreateJobProcessor :98-106
        const int64_t key = cmd.key < 0 ? job_keys.next_key() : cmd.key;
        job_states[key] = JS_CREATED;
        accept(JOB_CREATED, key);
        break;
      }
      case JOB_ACTIVATE:  // ActivateJobProcessor :108-160 (the push to the subscriber is a side effect)
        if (s0 == JS_CREATED || s0 == JS_FAILED || s0 == JS_TIMED_OUT) {
          job_states[cmd.key] = JS_ACTIVATED;
          accept(JOB_ACTIVATED, cmd.key);
        } else {
          write_rejection(cmd, REJ_NOT_APPLICABLE, "Job is not in one of these states: CREATED, FAILED, TIMED_OUT");
        }
        break;
      case JOB_COMPLETE:  // CompleteJobProcessor :162-175
        if (s0 == JS_ACTIVATED || s0 == JS_TIMED_OUT) {
          job_states.erase(cmd.key);
          accept(JOB_COMPLETED, cmd.key);
        } else {
          write_rejection(cmd, REJ_NOT_APPLICABLE, "Job is not in state: ACTIVATED, TIMED_OUT");
        }
        break;
      case JOB_FAIL:  // FailJobProcessor :177-189
        if (s0 == JS_ACTIVATED) { job_states[cmd.key] = JS_FAILED; accept(JOB_FAILED, cmd.key); }
        else write_rejection(cmd, REJ_NOT_APPLICABLE, "Job is not in state ACTIVATED");
        break;
      case JOB_TIME_OUT:  // TimeOutJobProcessor :191-204
        if (s0 == JS_ACTIVATED) { job_states[cmd.key] = JS_TIMED_OUT; accept(JOB_TIMED_OUT, cmd.key); }
        else write_rejection(cmd, REJ_NOT_APPLICABLE, "Job is not in state ACTIVATED");
        break;
      case JOB_UPDATE_RETRIES:  // UpdateRetriesJobProcessor :206-222
        if (s0 == JS_FAILED) {
          if (cmd.job.retries > 0) accept(JOB_RETRIES_UPDATED, cmd.key);
          else write_rejection(cmd, REJ_BAD_VALUE, "Retries must be greater than 0");
        } else {
          write_rejection(cmd, REJ_NOT_APPLICABLE, "Job is not in state FAILED");
        }
        break;
      case JOB_CANCEL:  // CancelJobProcessor :224-240
        if (s0 != JS_NONE) { job_states.erase(cmd.key); accept(JOB_CANCELED, cmd.key); }
        else write_rejection(cmd, REJ_NOT_APPLICABLE, "Job does not exist");
        break;
      default:
        break;
    }
  }

  // canonical harness: the job processor as a deterministic FIFO participant
  void harness_job_create(const Record& cmd) {
    int64_t job_key = job_keys.next_key();
    w_->new_batch();
    Record a = cmd;
    a.key = job_key; a.record_type = RT_EVENT; a.intent = JOB_CREATED;
    w_->stage(a);
    Record b = cmd;
    b.key = job_key; b.record_type = RT_EVENT; b.intent = JOB_COMPLETED;
    auto it = job_payloads.find({cmd.job.h_workflow_key, cmd.job.h_activity_id});
    b.job.payload = it == job_payloads.end() ? EMPTY_DOCUMENT : it->second;
    w_->stage(b);
  }

  // ---------------------------------------------------------------- BpmnStepProcessor :177-251
  void bpmn_step(const Record& rec) {
    Workflow* wf = by_key(rec.wf.workflow_key);
    if (!wf) throw ZbError("workflow not deployed");
    Element* el = wf->get(rec.wf.activity_id);
    ElementInstance* ei = index.get(rec.key);
    ElementInstance* scope = index.get(rec.wf.scope_instance_key);
    if (!ei && !scope) return;
    // step guards :128-150
    bool ok;
    switch (rec.intent) {
      case ELEMENT_READY: case ELEMENT_ACTIVATED: case ELEMENT_COMPLETING:
        if (!ei) throw ZbError("NullPointerException in noConcurrentTransitionGuard");
        ok = rec.intent == ei->state; break;
      case ELEMENT_COMPLETED: case END_EVENT_OCCURRED: case GATEWAY_ACTIVATED: case START_EVENT_OCCURRED:
      case SEQUENCE_FLOW_TAKEN:
        ok = scope && scope->state == ELEMENT_ACTIVATED; break;
      case ELEMENT_TERMINATING: ok = true; break;
      case ELEMENT_TERMINATED: ok = scope && scope->state == ELEMENT_TERMINATING; break;
      default: ok = false;
    }
    if (!ok) return;
    if (!el) throw ZbError("NullPointerException: unknown element");
    uint8_t step = el->get_step(rec.intent);
    if (step == S_UNBOUND || step == S_NONE) return;
    handle(step, rec, el, ei, scope, wf);
  }

  void handle(uint8_t step, const Record& rec, Element* el, ElementInstance* ei, ElementInstance* scope, Workflow* wf) {
    WfValue v = rec.wf;
    switch (step) {
      case S_APPLY_INPUT_MAPPING:  // InputMappingHandler :39-70
        if (!el->input_mappings.empty()) {
          try {
            v.set_payload(map_extract(v.payload, el->input_mappings));
          } catch (const MappingError& e) {
            raise_incident(rec, ERR_IO_MAPPING, e.what());
            break;
          }
        }
        write_followup_wf_event(rec.key, ELEMENT_ACTIVATED, v);
        break;
      case S_APPLY_OUTPUT_MAPPING: {  // OutputMappingHandler :42-85 (outputBehavior null => merge)
        if (el->output_behavior == Element::OB_NONE) {
          v.set_payload(scope->value.payload);
        } else {
          const bytes target = el->output_behavior == Element::OB_OVERWRITE ? EMPTY_DOCUMENT : scope->value.payload;
          try {
            v.set_payload(map_merge(v.payload, target, el->output_mappings));
          } catch (const MappingError& e) {
            raise_incident(rec, ERR_IO_MAPPING, e.what());
            break;
          }
        }
        write_followup_wf_event(rec.key, ELEMENT_COMPLETED, v);
        break;
      }
      case S_CREATE_JOB: {  // CreateJobHandler :33-56
        Record j;
        j.key = -1; j.record_type = RT_COMMAND; j.value_type = VT_JOB; j.intent = JOB_CREATE;
        j.job.type = el->job_type;
        j.job.retries = el->retries;
        j.job.payload = v.payload;
        j.job.h_bpmn_process_id = v.bpmn_process_id;
        j.job.h_version = v.version;
        j.job.h_workflow_key = v.workflow_key;
        j.job.h_workflow_instance_key = v.workflow_instance_key;
        j.job.h_activity_id = el->id;
        j.job.h_activity_instance_key = rec.key;
        j.job.custom_headers = el->encoded_headers;
        w_->stage(std::move(j));
        break;
      }
      case S_EXCLUSIVE_SPLIT: {  // ExclusiveSplitHandler :38-71
        Element* chosen = nullptr;
        try {
          for (Element* f : el->outgoing_with_condition) {
            if (interp_.eval(f->condition->root.get(), (const uint8_t*)v.payload.data(), v.payload.size())) {
              chosen = f;
              break;
            }
          }
          if (!chosen) chosen = el->default_flow;
        } catch (const ConditionError& e) {
          raise_incident(rec, ERR_CONDITION, e.what());
          break;
        }
        if (chosen) {
          v.activity_id = chosen->id;
          write_new_wf_event(SEQUENCE_FLOW_TAKEN, v);
        } else {
          raise_incident(rec, ERR_CONDITION, "All conditions evaluated to false and no default flow is set.");
        }
        break;
      }
      case S_CONSUME_TOKEN: {  // ConsumeTokenHandler :30-43
        // EXTENSION (C4): with parallel gateways a scope holds several tokens and completes when its
        // last token is consumed. Without them every scope holds exactly one token here (tokens == 1),
        // so this is the reference's unconditional completion.
        if (--scope->tokens > 0) break;
        WfValue sv = scope->value;
        sv.payload = v.payload;
        write_followup_wf_event(v.scope_instance_key, ELEMENT_COMPLETING, sv);
        break;
      }
      case S_PARALLEL_SPLIT: {  // EXTENSION (C4): fork, one SEQUENCE_FLOW_TAKEN per outgoing flow
        // executable (reverse document) order; the join arity merges incoming tokens into one
        scope->tokens += (int32_t)el->outgoing.size() - std::max(el->incoming, 1);
        w_->new_batch();
        for (Element* f : el->outgoing) {
          WfValue fv = v;
          fv.activity_id = f->id;
          write_new_wf_event(SEQUENCE_FLOW_TAKEN, fv);
        }
        break;
      }
      case S_PARALLEL_MERGE: {  // EXTENSION (C4): join, fires on the arrival that completes the arity
        Element* gw = el->target;
        int32_t& n = scope->joins[gw];
        if (++n < gw->incoming) break;
        n = 0;
        v.activity_id = gw->id;
        write_new_wf_event(GATEWAY_ACTIVATED, v);
        break;
      }
      case S_TAKE_SEQUENCE_FLOW:  // TakeSequenceFlowHandler :30-38
        v.activity_id = el->outgoing.at(0)->id;
        write_new_wf_event(SEQUENCE_FLOW_TAKEN, v);
        break;
      case S_ACTIVATE_GATEWAY:
        v.activity_id = el->target->id;
        write_new_wf_event(GATEWAY_ACTIVATED, v);
        break;
      case S_START_STATEFUL_ELEMENT:
        v.activity_id = el->target->id;
        write_new_wf_event(ELEMENT_READY, v);
        break;
      case S_TRIGGER_END_EVENT:
        v.activity_id = el->target->id;
        write_new_wf_event(END_EVENT_OCCURRED, v);
        break;
      case S_TRIGGER_START_EVENT:  // TriggerStartEventHandler :30-39
        if (!el->start_event) throw ZbError("NullPointerException: container without start event");
        v.activity_id = el->start_event->id;
        v.scope_instance_key = rec.key;
        ei->tokens = 1;  // EXTENSION (C4): the start event's token
        write_new_wf_event(START_EVENT_OCCURRED, v);
        break;
      case S_COMPLETE_PROCESS:  // CompleteProcessHandler :28-35
        write_followup_wf_event(rec.key, ELEMENT_COMPLETED, v);
        break;
      case S_SUBSCRIBE_TO_INTERMEDIATE_MESSAGE: {  // SubscribeMessageHandler :77-141
        jp_.run(el->correlation_key.filters, (const uint8_t*)v.payload.data(), v.payload.size());
        if (jp_.results.size() != 1) throw ZbError("Failed to extract correlation-key: no result");
        MpReader r((const uint8_t*)v.payload.data() + jp_.results[0].position, jp_.results[0].length);
        MpToken t = r.read_token();
        bytes ck;
        if (t.type == MpType::STRING) ck = t.value();
        else if (t.type == MpType::INTEGER) {
          ck.resize(8);  // UnsafeBuffer.putLong: native (little endian) byte order
          uint64_t u = (uint64_t)t.ival;
          for (int i = 0; i < 8; i++) ck[i] = (char)((u >> (8 * i)) & 0xff);
        } else throw ZbError("Failed to extract correlation-key: wrong type");
        int32_t h = 0;  // SubscriptionUtil.getSubscriptionHashCode (signed bytes)
        for (char c : ck) h = (int32_t)((uint32_t)h * 31u + (uint32_t)(int32_t)(int8_t)c);
        int32_t part = h % partition_count;
        if (part < 0) part = -part;
        side_effects.push_back({1, v.workflow_instance_key, rec.key, el->message_name, ck, part, partition_id, bytes()});
        break;
      }
      case S_TERMINATE_ELEMENT:
      case S_TERMINATE_JOB_TASK: {  // TerminateElementHandler / TerminateServiceTaskHandler
        w_->new_batch();
        if (step == S_TERMINATE_JOB_TASK && ei && ei->job_key > 0) {
          Record j;
          j.key = ei->job_key; j.record_type = RT_COMMAND; j.value_type = VT_JOB; j.intent = JOB_CANCEL;
          j.job.type = bytes();
          j.job.h_bpmn_process_id = v.bpmn_process_id;
          j.job.h_version = v.version;
          j.job.h_workflow_instance_key = v.workflow_instance_key;
          j.job.h_activity_id = v.activity_id;
          j.job.h_activity_instance_key = ei->key;
          w_->stage(std::move(j));
        }
        write_followup_wf_event(rec.key, ELEMENT_TERMINATED, v);
        break;
      }
      case S_TERMINATE_CONTAINED_INSTANCES: {  // TerminateContainedElementsHandler :31-53
        if (ei->children.empty()) {
          write_followup_wf_event(rec.key, ELEMENT_TERMINATED, v);
        } else {
          ElementInstance* child = ei->children[0];
          if (child->state == ELEMENT_READY || child->state == ELEMENT_ACTIVATED || child->state == ELEMENT_COMPLETING)
            write_followup_wf_event(child->key, ELEMENT_TERMINATING, child->value);
        }
        break;
      }
      case S_PROPAGATE_TERMINATION:  // PropagateTerminationHandler :29-40
        if (scope->children.empty()) {
          write_followup_wf_event(scope->key, ELEMENT_TERMINATED, scope->value);
        } else {
          // EXTENSION (C4, several live tokens in one scope; unreachable in the reference, where a
          // scope has at most one child): terminate the next child, as TerminateContainedElementsHandler
          // does for the first one.
          ElementInstance* child = scope->children[0];
          if (child->state == ELEMENT_READY || child->state == ELEMENT_ACTIVATED || child->state == ELEMENT_COMPLETING)
            write_followup_wf_event(child->key, ELEMENT_TERMINATING, child->value);
        }
        break;
      default:
        break;
    }
    (void)wf;
  }
};

}  // namespace zbref


// =============================================================================== C API (ctypes)
using namespace zbref;

// ------------------------------------------------------------------------------ log frames (§8f rank 1)
// One record as LogStreamBatchWriterImpl.writeEventsToBuffer (:222-268) / LogStreamWriterImpl.tryWrite lay it
// into the dispatcher buffer: DataFrameDescriptor header (:53-96, 12 B: framed length, version, flags, type
// TYPE_MESSAGE, stream id = partition id), LogEntryDescriptor header (:28-121, 48 B), RecordMetadata
// (RecordMetadata.java:96-128: SBE message header + 34-byte block + varData rejectionReason, protocol.xml:135-146),
// the value, zero padding to FRAME_ALIGNMENT 8. Position: the record's log position (the dispatcher would
// derive it from the byte offset of the claim; the caller maps it).
static void put_le(bytes& b, uint64_t v, int n) {
  for (int i = 0; i < n; i++) b.push_back((char)(uint8_t)(v >> (8 * i)));
}
bytes encode_frame(const Record& r, int32_t stream_id, int32_t raft_term, int64_t timestamp) {
  const bytes v = r.encode_value();
  const std::string& reason = r.record_type == RT_REJECTION ? r.rejection_reason : std::string();
  const uint32_t meta_len = 8 + 34 + 2 + (uint32_t)reason.size();
  const uint32_t framed = 12 + 48 + meta_len + (uint32_t)v.size();
  bytes b;
  b.reserve((framed + 7) & ~7u);
  put_le(b, framed, 4);
  put_le(b, 0, 1);                 // version
  put_le(b, r.batch_flags, 1);
  put_le(b, 0, 2);                 // TYPE_MESSAGE
  put_le(b, (uint32_t)stream_id, 4);
  put_le(b, 0, 2);                 // LogEntryDescriptor version
  put_le(b, 0, 2);                 // reserved
  put_le(b, (uint64_t)r.position, 8);
  put_le(b, (uint32_t)raft_term, 4);
  put_le(b, (uint32_t)r.producer_id, 4);
  put_le(b, (uint64_t)r.source_position, 8);
  put_le(b, (uint64_t)r.key, 8);
  put_le(b, (uint64_t)timestamp, 8);
  put_le(b, meta_len, 2);
  put_le(b, 0, 2);                 // unused
  put_le(b, 34, 2);                // SBE header: blockLength, templateId 200, schemaId 0, version 1
  put_le(b, 200, 2);
  put_le(b, 0, 2);
  put_le(b, 1, 2);
  put_le(b, r.record_type, 1);
  put_le(b, (uint32_t)r.request_stream_id, 4);
  put_le(b, r.request_id, 8);
  put_le(b, UINT64_MAX, 8);        // subscriptionId (null)
  put_le(b, 1, 2);                 // protocolVersion = Protocol.PROTOCOL_VERSION
  put_le(b, r.value_type, 1);
  put_le(b, r.intent, 1);
  put_le(b, UINT64_MAX, 8);        // incidentKey (null)
  put_le(b, r.rejection_type, 1);
  put_le(b, reason.size(), 2);
  b.append(reason);
  b.append(v);
  while (b.size() & 7) b.push_back(0);
  return b;
}


struct zbref_record {
  int64_t position;
  int64_t source_position;
  int64_t key;
  uint8_t record_type;
  uint8_t value_type;
  uint8_t intent;
  uint8_t rejection_type;
  uint32_t value_len;
};

// The CPU baseline runs one oracle partition per thread. glibc's defaults (arenas grown and trimmed in small
// steps, large vectors from mmap) put every partition's page faults and mprotect / munmap calls under the
// process-wide mmap lock: 8 threads ran C1 as slowly as 1.5 threads' worth. Large arena steps, no trimming and
// large vectors from the arena (with an untimed warm-up run per thread, bench.py) let them scale.
__attribute__((constructor)) static void zbref_malloc_tuning() {
  mallopt(M_MMAP_THRESHOLD, 32 << 20);
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
  mallopt(M_TOP_PAD, 64 << 20);
}

extern "C" {

void* zbref_new(int partition_id, int partition_count) {
  auto* e = new Engine();
  e->partition_id = partition_id;
  e->partition_count = partition_count;
  return e;
}
void zbref_free(void* h) { delete (Engine*)h; }

const char* zbref_last_error(void* h) { return ((Engine*)h)->last_error.c_str(); }

int zbref_deploy(void* h, const char* xml, size_t len, int64_t workflow_key, int32_t version) {
  Engine* e = (Engine*)h;
  try {
    e->deploy(std::string(xml, len), workflow_key, version);
    return 0;
  } catch (const std::exception& ex) {
    e->last_error = ex.what();
    return -1;
  }
}

int zbref_set_job_payload(void* h, int64_t workflow_key, const char* activity_id, const uint8_t* p, size_t n) {
  Engine* e = (Engine*)h;
  e->job_payloads[{workflow_key, bytes(activity_id)}] = bytes((const char*)p, n);
  return 0;
}

int zbref_submit_create(void* h, const char* process_id, int32_t version, int64_t workflow_key, const uint8_t* p,
                        size_t n) {
  Engine* e = (Engine*)h;
  try {
    e->submit_create(bytes(process_id), version, workflow_key, bytes((const char*)p, n));
    return 0;
  } catch (const std::exception& ex) {
    e->last_error = ex.what();
    return -1;
  }
}

int zbref_set_harness(void* h, int on) {
  ((Engine*)h)->harness = on != 0;
  return 0;
}

// the job stream processor on (harness off): JOB commands go through JobInstanceStreamProcessor
int zbref_set_job_processor(void* h, int on) {
  Engine* e = (Engine*)h;
  e->job_processor = on != 0;
  if (on) e->harness = false;
  return 0;
}

int zbref_submit_record(void* h, uint8_t record_type, uint8_t value_type, uint8_t intent, int64_t key,
                        const uint8_t* value, size_t n) {
  Engine* e = (Engine*)h;
  try {
    e->submit_record(record_type, value_type, intent, key, bytes((const char*)value, n));
    return 0;
  } catch (const std::exception& ex) {
    e->last_error = ex.what();
    return -1;
  }
}

// Live element instances sorted by key (ElementInstanceIndex.java:25-65): per instance
// [i64 key][i64 parent key (-1)][i64 job key][u8 state][3 pad][u32 value length][value bytes].
int64_t zbref_dump_instances(void* h, uint8_t* buf, size_t cap) {
  Engine* e = (Engine*)h;
  std::vector<const ElementInstance*> v;
  for (auto& kv : e->index.instances) v.push_back(kv.second.get());
  std::sort(v.begin(), v.end(), [](const ElementInstance* a, const ElementInstance* b) { return a->key < b->key; });
  size_t off = 0;
  for (const ElementInstance* ei : v) {
    bytes val = ei->value.encode();
    size_t need = 32 + val.size();
    if (buf && off + need <= cap) {
      int64_t pk = ei->parent ? ei->parent->key : -1;
      std::memcpy(buf + off, &ei->key, 8);
      std::memcpy(buf + off + 8, &pk, 8);
      std::memcpy(buf + off + 16, &ei->job_key, 8);
      buf[off + 24] = ei->state;
      buf[off + 25] = buf[off + 26] = buf[off + 27] = 0;
      uint32_t n = (uint32_t)val.size();
      std::memcpy(buf + off + 28, &n, 4);
      std::memcpy(buf + off + 32, val.data(), val.size());
    }
    off += need;
  }
  return (int64_t)off;
}

// bulk form of zbref_submit_create: n payloads, offsets[n + 1] into blob
int zbref_submit_creates(void* h, const char* process_id, int32_t version, int64_t workflow_key, size_t n,
                         const uint8_t* blob, const uint64_t* offsets) {
  Engine* e = (Engine*)h;
  try {
    const bytes pid(process_id);
    for (size_t i = 0; i < n; i++)
      e->submit_create(pid, version, workflow_key, bytes((const char*)blob + offsets[i], offsets[i + 1] - offsets[i]));
    return 0;
  } catch (const std::exception& ex) {
    e->last_error = ex.what();
    return -1;
  }
}

int zbref_submit_cancel(void* h, int64_t key) {
  ((Engine*)h)->submit_cancel(key);
  return 0;
}

int zbref_submit_open(void* h, int32_t wfp, int64_t wik, int64_t aik, const uint8_t* name, size_t nn,
                      const uint8_t* ck, size_t nck) {
  ((Engine*)h)->submit_open(wfp, wik, aik, bytes((const char*)name, nn), bytes((const char*)ck, nck));
  return 0;
}

int zbref_submit_publish(void* h, const uint8_t* name, size_t nn, const uint8_t* ck, size_t nck, int64_t ttl,
                         const uint8_t* p, size_t np, const uint8_t* id, size_t nid) {
  ((Engine*)h)->submit_publish(bytes((const char*)name, nn), bytes((const char*)ck, nck), ttl,
                               bytes((const char*)p, np), bytes((const char*)id, nid));
  return 0;
}

// ActorClock for the message stream processor (deadline = timeToLive + now, MessageDataStore.Message)
int zbref_set_clock(void* h, int64_t now_ms) {
  ((Engine*)h)->clock_ms = now_ms;
  return 0;
}
// MessageTimeToLiveChecker.run at now_ms: appends the DELETE commands (processed by the next run)
int64_t zbref_check_ttl(void* h, int64_t now_ms) { return (int64_t)((Engine*)h)->check_ttl(now_ms); }

int64_t zbref_side_effect_count(void* h) { return (int64_t)((Engine*)h)->side_effects.size(); }

// kind/partition/wf_partition + keys; byte fields copied when their capacity (4096 each) suffices
int zbref_side_effect_get(void* h, int64_t i, int32_t* ints, int64_t* keys, uint8_t* name, uint8_t* ck,
                          uint8_t* payload, uint64_t* lens) {
  const SideEffect& s = ((Engine*)h)->side_effects.at((size_t)i);
  ints[0] = s.kind; ints[1] = s.partition; ints[2] = s.wf_partition;
  keys[0] = s.workflow_instance_key; keys[1] = s.activity_instance_key;
  const bytes* f[3] = {&s.message_name, &s.correlation_key, &s.payload};
  uint8_t* d[3] = {name, ck, payload};
  for (int k = 0; k < 3; k++) {
    lens[k] = f[k]->size();
    if (f[k]->size() <= 4096) std::memcpy(d[k], f[k]->data(), f[k]->size());
  }
  return 0;
}

void zbref_clear_side_effects(void* h) { ((Engine*)h)->side_effects.clear(); }

int zbref_submit_correlate(void* h, int64_t wik, int64_t aik, const char* name, const uint8_t* p, size_t n) {
  ((Engine*)h)->submit_correlate(wik, aik, bytes(name), bytes((const char*)p, n));
  return 0;
}

// Process until the log is exhausted (quiescence) or max records; returns #processed or -1.
int64_t zbref_run(void* h, int64_t max_records) {
  Engine* e = (Engine*)h;
  try {
    return (int64_t)e->run(max_records < 0 ? SIZE_MAX : (size_t)max_records);
  } catch (const std::exception& ex) {
    if (e->last_error.empty()) e->last_error = ex.what();
    return -1;
  }
}

// request metadata of a submitted command (the client API's requestId / requestStreamId)
// positions of the API below are log positions: log[position - pos_base]
int zbref_set_position_base(void* h, int64_t base) {
  Engine* e = (Engine*)h;
  if (!e->log.empty() || base < 0) return -1;
  e->pos_base = base;
  return 0;
}

int zbref_set_request(void* h, int64_t position, uint64_t request_id, int32_t request_stream_id) {
  Engine* e = (Engine*)h;
  position -= e->pos_base;
  if (position < 0 || position >= (int64_t)e->log.size()) return -1;
  e->log[(size_t)position].request_id = request_id;
  e->log[(size_t)position].request_stream_id = request_stream_id;
  return 0;
}

// log frames of records [from, to), contiguous; returns the byte count (written when it fits cap)
int64_t zbref_frames(void* h, int64_t from, int64_t to, int32_t stream_id, int32_t raft_term, int64_t timestamp,
                     uint8_t* buf, size_t cap) {
  Engine* e = (Engine*)h;
  from = std::max<int64_t>(from - e->pos_base, 0);
  to = to < 0 ? (int64_t)e->log.size() : to - e->pos_base;
  if (to > (int64_t)e->log.size()) to = (int64_t)e->log.size();
  size_t off = 0;
  for (int64_t i = from; i < to; i++) {
    const bytes f = encode_frame(e->log[(size_t)i], stream_id, raft_term, timestamp);
    if (buf && off + f.size() <= cap) std::memcpy(buf + off, f.data(), f.size());
    off += f.size();
  }
  return (int64_t)off;
}

int64_t zbref_log_size(void* h) { return ((Engine*)h)->pos_base + (int64_t)((Engine*)h)->log.size(); }

// Fills header and returns the encoded value into buf (if cap suffices); returns value length.
int64_t zbref_get_record(void* h, int64_t i, zbref_record* out, uint8_t* buf, size_t cap) {
  Engine* e = (Engine*)h;
  const Record& r = e->log.at((size_t)(i - e->pos_base));
  bytes v = r.encode_value();
  out->position = r.position;
  out->source_position = r.source_position;
  out->key = r.key;
  out->record_type = r.record_type;
  out->value_type = r.value_type;
  out->intent = r.intent;
  out->rejection_type = r.rejection_type;
  out->value_len = (uint32_t)v.size();
  if (buf && v.size() <= cap) std::memcpy(buf, v.data(), v.size());
  return (int64_t)v.size();
}

// Writes the whole log as a flat buffer: per record [zbref_record][value bytes].
int64_t zbref_dump_log(void* h, int64_t from, int64_t to, uint8_t* buf, size_t cap) {
  Engine* e = (Engine*)h;
  size_t off = 0;
  from = std::max<int64_t>(from - e->pos_base, 0);
  to = to < 0 ? (int64_t)e->log.size() : to - e->pos_base;
  if (to > (int64_t)e->log.size()) to = (int64_t)e->log.size();
  for (int64_t i = from; i < to; i++) {
    const Record& r = e->log[(size_t)i];
    bytes v = r.encode_value();
    size_t need = sizeof(zbref_record) + v.size();
    if (buf && off + need <= cap) {
      zbref_record hr{r.position, r.source_position, r.key, r.record_type, r.value_type, r.intent, r.rejection_type,
                      (uint32_t)v.size()};
      std::memcpy(buf + off, &hr, sizeof(hr));
      std::memcpy(buf + off + sizeof(hr), v.data(), v.size());
    }
    off += need;
  }
  return (int64_t)off;
}

void zbref_counters(void* h, int64_t* out) {
  Engine* e = (Engine*)h;
  out[0] = e->created;
  out[1] = e->completed;
  out[2] = e->canceled;
  out[3] = (int64_t)e->index.instances.size();
  out[4] = e->wf_keys.next;
  out[5] = e->job_keys.next;
  out[6] = e->transitions;
}

int64_t zbref_side_effects(void* h, int64_t i, int64_t* keys, int32_t* partition, uint8_t* ck, size_t cap) {
  Engine* e = (Engine*)h;
  if (i < 0) return (int64_t)e->side_effects.size();
  const SideEffect& s = e->side_effects.at((size_t)i);
  keys[0] = s.workflow_instance_key;
  keys[1] = s.activity_instance_key;
  *partition = s.partition;
  if (s.correlation_key.size() <= cap) std::memcpy(ck, s.correlation_key.data(), s.correlation_key.size());
  return (int64_t)s.correlation_key.size();
}

// ---- unit-level entry points for the reference's known-answer tests
// returns 1/0 for true/false, -1 compile error, -2 evaluation error (message in err)
int zbref_eval_condition(const char* expr, const uint8_t* doc, size_t n, char* err, size_t errcap) {
  CompiledCondition c = create_condition(expr);
  if (!c.valid) {
    std::snprintf(err, errcap, "%s", c.error.c_str());
    return -1;
  }
  ElInterpreter in;
  try {
    return in.eval(c.root.get(), doc, n) ? 1 : 0;
  } catch (const std::exception& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -2;
  }
}

// Evaluate one compiled condition against several documents in sequence (constant mutation persists).
int zbref_eval_condition_seq(const char* expr, const uint8_t* docs, const uint32_t* lens, int ndocs, int* results) {
  CompiledCondition c = create_condition(expr);
  if (!c.valid) return -1;
  ElInterpreter in;
  size_t off = 0;
  for (int i = 0; i < ndocs; i++) {
    try {
      results[i] = in.eval(c.root.get(), docs + off, lens[i]) ? 1 : 0;
    } catch (const std::exception&) {
      results[i] = -2;
    }
    off += lens[i];
  }
  return 0;
}

int64_t zbref_merge(const uint8_t* src, size_t ns, const uint8_t* tgt, size_t nt, uint8_t* out, size_t cap, char* err,
                    size_t errcap) {
  try {
    bytes r = merge_documents(bytes((const char*)src, ns), bytes((const char*)tgt, nt));
    if (r.size() <= cap) std::memcpy(out, r.data(), r.size());
    return (int64_t)r.size();
  } catch (const std::exception& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -1;
  }
}

// MappingProcessor.extract (tgt == nullptr) / merge with explicit mappings; mappings = "source\ttarget\n"...
// returns the result length, -1 MappingException (err has its message), -2 any other failure
int64_t zbref_map(const uint8_t* src, size_t ns, const uint8_t* tgt, size_t nt, const char* mappings, uint8_t* out,
                  size_t cap, char* err, size_t errcap) {
  try {
    std::vector<Mapping> ms;
    JsonPathCompiler jc;
    std::string all(mappings);
    size_t p = 0;
    while (p < all.size()) {
      size_t nl = all.find('\n', p);
      if (nl == std::string::npos) nl = all.size();
      std::string line = all.substr(p, nl - p);
      size_t tab = line.find('\t');
      if (tab != std::string::npos) ms.push_back({jc.compile(line.substr(0, tab)), line.substr(tab + 1)});
      p = nl + 1;
    }
    bytes s((const char*)src, ns);
    bytes r = tgt ? map_merge(s, bytes((const char*)tgt, nt), ms) : map_extract(s, ms);
    if (r.size() <= cap) std::memcpy(out, r.data(), r.size());
    return (int64_t)r.size();
  } catch (const MappingError& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -1;
  } catch (const std::exception& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -2;
  }
}

// MsgPackTree as MsgPackDocumentIndexer.index (mode 0) or MsgPackDocumentExtractor.extract (mode 1, mappings
// "source\ttarget\n"...) builds it for doc, in the dump format of tests/native/devlib_host.cpp devlib_xtree_dump (nodes
// sorted by id here). Returns the dump length, -1 MappingException / -2 other failure (err has the message).
int64_t zbref_tree_dump(const uint8_t* doc, size_t n, const char* mappings, int mode, char* out, size_t cap, char* err,
                        size_t errcap) {
  try {
    bytes d((const char*)doc, n);
    MsgPackTree t;
    if (mode == 0) {
      DocumentIndexer ix;
      ix.index(t, d);
    } else {
      std::vector<Mapping> ms;
      JsonPathCompiler jc;
      std::string all(mappings);
      size_t p = 0;
      while (p < all.size()) {
        size_t nl = all.find('\n', p);
        if (nl == std::string::npos) nl = all.size();
        std::string line = all.substr(p, nl - p);
        size_t tab = line.find('\t');
        if (tab != std::string::npos) ms.push_back({jc.compile(line.substr(0, tab)), line.substr(tab + 1)});
        p = nl + 1;
      }
      extract_mappings(t, d, ms);
    }
    std::vector<std::string> ids;
    for (auto& kv : t.node_type) ids.push_back(kv.first);
    std::sort(ids.begin(), ids.end());
    std::string o;
    static const char HEX[] = "0123456789abcdef";
    for (auto& id : ids) {
      const NodeType nt = t.node_type.at(id);
      o += nt == NodeType::MAP ? 'M' : nt == NodeType::ARRAY ? 'A' : nt == NodeType::EXTRACTED_LEAF ? 'X' : 'L';
      o += '\0';
      o += id;
      o += '\0';
      auto c = t.childs.find(id);
      if (c != t.childs.end())
        for (size_t k = 0; k < c->second.order.size(); k++) {
          if (k) o += '\x1e';
          o += c->second.order[k];
        }
      o += '\0';
      auto l = t.leaf.find(id);
      if (l != t.leaf.end()) {
        const uint32_t pos = (uint32_t)(l->second >> 32), len = (uint32_t)l->second;
        for (uint32_t k = 0; k < len; k++) { o += HEX[(uint8_t)d[pos + k] >> 4]; o += HEX[(uint8_t)d[pos + k] & 15]; }
      }
      o += '\n';
    }
    if (o.size() <= cap) std::memcpy(out, o.data(), o.size());
    return (int64_t)o.size();
  } catch (const MappingError& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -1;
  } catch (const std::exception& ex) {
    std::snprintf(err, errcap, "%s", ex.what());
    return -2;
  }
}

// returns #results (positions/lengths written pairwise), -1 invalid query (err has message)
int zbref_query(const char* path, const uint8_t* doc, size_t n, int32_t* out, int cap, char* err, size_t errcap) {
  JsonPathCompiler jc;
  JsonPathQuery q = jc.compile(path);
  if (!q.valid()) {
    std::snprintf(err, errcap, "%s", q.error.c_str());
    return -1;
  }
  JsonPathExecutor ex;
  ex.run(q.filters, doc, n);
  int k = 0;
  for (auto& r : ex.results) {
    if (k < cap) { out[2 * k] = r.position; out[2 * k + 1] = r.length; }
    k++;
  }
  return k;
}

// JsonPathTokenizer.tokenize: (token, position, length) triples in visit order, token = JpToken's enum index
int zbref_jp_tokens(const char* expr, int32_t* out, int cap) {
  int k = 0;
  jp_tokenize(bytes(expr), [&](JpToken t, int off, int len) {
    if (k < cap) { out[3 * k] = (int32_t)t; out[3 * k + 1] = off; out[3 * k + 2] = len; }
    k++;
  });
  return k;
}

// JsonPathQueryCompiler.compile: the filter instances (filter id, index) -- #instances, or -1 for an invalid query
// with its invalid position and error reason (JsonPathQuery.getInvalidPosition / getErrorReason)
int zbref_jp_compile(const char* expr, int32_t* ids, int32_t* idx, int cap, int32_t* invalid_pos, char* err,
                     size_t errcap) {
  JsonPathCompiler jc;
  JsonPathQuery q = jc.compile(bytes(expr));
  *invalid_pos = q.invalid_position;
  if (!q.valid()) {
    std::snprintf(err, errcap, "%s", q.error.c_str());
    return -1;
  }
  int k = 0;
  for (auto& f : q.filters) {
    if (k < cap) { ids[k] = f.id; idx[k] = f.index; }
    k++;
  }
  return k;
}

// MsgPackReader.readToken on p[0, n): out = type (MpType index), boolean, size, value offset, value length, bytes
// consumed; 0, or -1 with the reader's exception message
int zbref_read_token(const uint8_t* p, size_t n, int64_t* ival, double* fval, int32_t* out, char* err, size_t errcap) {
  MpReader r(p, n);
  try {
    MpToken t = r.read_token();
    *ival = t.ival;
    *fval = t.fval;
    out[0] = (int32_t)t.type; out[1] = t.bval ? 1 : 0; out[2] = (int32_t)t.size;
    out[3] = t.data ? (int32_t)(t.data - p) : -1; out[4] = (int32_t)t.len; out[5] = (int32_t)r.off;
    return 0;
  } catch (const std::exception& e) {
    std::snprintf(err, errcap, "%s", e.what());
    return -1;
  }
}

// MsgPackTraverser.traverse: 1 when every token reads; 0 with getInvalidPosition / getErrorMessage otherwise
int zbref_traverse(const uint8_t* doc, size_t n, int32_t* invalid_pos, char* err, size_t errcap) {
  MpReader r(doc, n);
  *invalid_pos = -1;
  while (r.has_next()) {
    const size_t pos = r.off;
    try {
      (void)r.read_token();
    } catch (const std::exception& e) {
      *invalid_pos = (int32_t)pos;
      std::snprintf(err, errcap, "%s", e.what());
      return 0;
    }
  }
  return 1;
}

int32_t zbref_subscription_hash(const uint8_t* p, size_t n) {
  int32_t h = 0;
  for (size_t i = 0; i < n; i++) h = (int32_t)((uint32_t)h * 31u + (uint32_t)(int32_t)(int8_t)p[i]);
  return h;
}

int64_t zbref_encode_int(int64_t v, uint8_t* out) {
  MpWriter w;
  w.integer(v);
  std::memcpy(out, w.b.data(), w.b.size());
  return (int64_t)w.b.size();
}

int64_t zbref_encode_float(double v, uint8_t* out) {
  MpWriter w;
  w.floating(v);
  std::memcpy(out, w.b.data(), w.b.size());
  return (int64_t)w.b.size();
}

// Wall-clock timing helper for the CPU baseline: run to quiescence, return seconds.
// C5 CPU baseline (bench.py --config c5, cpu_baseline): P oracle partitions, each stepped on its own thread, with
// the exchange of zeebe_amd.cluster.LocalCluster.settle restated here (no Python in the timed region): run every
// partition to quiescence; if any emitted OPEN side effects, deliver them (per target partition: sources in
// partition order, emission order within a source) and repeat; else the same for CORRELATE; else done.
// Workload: n instances per partition of the deployed message workflow, instance i on partition
// i % P with payload {orderId: "order-<i>"}; then PUBLISH name "order", correlation key "order-<i>", payload
// {paid: true} on partition abs(hash % P). out: [0] wall seconds, [1] transitions, [2] completed, [3] rounds.
int zbref_c5_bench(int P, int64_t n, const char* xml, size_t xml_len, double* out) {
  std::vector<Engine*> parts;
  for (int p = 0; p < P; p++) parts.push_back((Engine*)zbref_new(p, P));
  for (Engine* e : parts)
    if (zbref_deploy(e, xml, xml_len, 100, 1) != 0) return -1;
  struct Fx { std::vector<SideEffect> v; };
  std::vector<Fx> fx(P);
  int64_t rounds = 0;
  bool failed = false;
  auto run_all = [&]() {
    std::vector<std::thread> ts;
    for (int p = 0; p < P; p++)
      ts.emplace_back([&, p]() {
        if (zbref_run(parts[p], -1) < 0) failed = true;
        for (auto& f : parts[p]->side_effects) fx[p].v.push_back(f);
        parts[p]->side_effects.clear();
      });
    for (auto& t : ts) t.join();
  };
  auto settle = [&]() {
    for (;;) {
      run_all();
      rounds++;
      if (failed) return;
      for (int kind = 1; kind <= 2; kind++) {
        bool any = false;
        for (int p = 0; p < P && !any; p++)
          for (auto& f : fx[p].v) any |= f.kind == kind;
        if (!any) continue;
        for (int q = 0; q < P; q++)
          for (int p = 0; p < P; p++)
            for (auto& f : fx[p].v)
              if (f.kind == kind && f.partition == q) {
                if (kind == 1) parts[q]->submit_open(f.wf_partition, f.workflow_instance_key, f.activity_instance_key,
                                                    f.message_name, f.correlation_key);
                else parts[q]->submit_correlate(f.workflow_instance_key, f.activity_instance_key, f.message_name,
                                                f.payload);
              }
        for (int p = 0; p < P; p++) {
          std::vector<SideEffect> rest;
          for (auto& f : fx[p].v)
            if (f.kind != kind) rest.push_back(f);
          fx[p].v.swap(rest);
        }
        goto next;
      }
      return;
    next:;
    }
  };
  auto mp_str = [](const std::string& s) {
    bytes b;
    if (s.size() < 32) b.push_back((char)(0xa0 | s.size()));
    else { b.push_back((char)0xd9); b.push_back((char)s.size()); }
    b += s;
    return b;
  };
  const bytes paid = std::string("\x81\xa4paid\xc3", 7);
  const int64_t N = n * P;
  const auto t0 = std::chrono::steady_clock::now();
  try {
    for (int64_t i = 0; i < N; i++)
      parts[i % P]->submit_create("msg", -1, -1, std::string("\x81\xa7orderId", 9) + mp_str("order-" + std::to_string(i)));
  } catch (const std::exception&) {
    failed = true;
  }
  if (!failed) settle();
  for (int64_t i = 0; i < N && !failed; i++) {
    const std::string ck = "order-" + std::to_string(i);
    const int32_t h = zbref_subscription_hash((const uint8_t*)ck.data(), ck.size());
    const int q = std::abs((int)(h % P));  // abs(hash % P), Java's remainder (SubscriptionCommandSender.java:105-109)
    parts[q]->submit_publish("order", ck, 3600000, paid, bytes());
  }
  if (!failed) settle();
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int64_t tr = 0, comp = 0, c[16];
  for (Engine* e : parts) {
    zbref_counters(e, c);
    tr += c[6];
    comp += c[1];
  }
  out[0] = wall; out[1] = (double)tr; out[2] = (double)comp; out[3] = (double)rounds;
  for (Engine* e : parts) zbref_free(e);
  return failed ? -1 : 0;
}

double zbref_run_timed(void* h, int64_t* processed) {
  auto t0 = std::chrono::steady_clock::now();
  int64_t n = zbref_run(h, -1);
  auto t1 = std::chrono::steady_clock::now();
  *processed = n;
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
