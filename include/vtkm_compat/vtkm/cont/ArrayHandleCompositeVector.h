// vtkm/cont/ArrayHandleCompositeVector.h: the VTK-m / reference name main.cc includes, over the librtp C ABI
// (include/rtp/vtkm_compat.hpp).
#pragma once
#include <rtp/vtkm_compat.hpp>
