// Band backend plugin API (stand-in; band/interface/tensor_view.h:37).
#pragma once
#include "band/interface/backend.h"
#include "band/interface/tensor.h"

namespace band {
namespace interface {
struct ITensorView : public IBackendSpecific, public ITensor {};
}  // namespace interface
}  // namespace band
