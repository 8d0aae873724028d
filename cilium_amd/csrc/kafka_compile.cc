// kafka_compile.cc — placeholder, replaced by the Kafka compiler.
#include "l7m_internal.h"
namespace l7m {
CompileResult compile_kafka(const l7m_kafka_rule*, size_t, const l7m_opts&) {
  CompileResult r;
  r.status = L7M_EUNSUPPORTED;
  r.err = "kafka not built yet";
  return r;
}
}  // namespace l7m
