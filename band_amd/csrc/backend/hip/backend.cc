#include "backend/hip/backend.h"

namespace band {

bool HipRegisterCreators() {
  BackendFactory::RegisterBackendCreators(BackendType::kTfLite, new hip::ModelExecutorCreator,
                                          new hip::ModelCreator, new hip::UtilCreator);
  return true;
}

// Strong definition of the symbol Band's factory references weakly.
bool TfLiteRegisterCreators() { return HipRegisterCreators(); }

}  // namespace band
