// vtkm/cont/ArrayHandleCounting.h: the VTK-m / reference name CornellBox.cpp includes, over the librtp C ABI
// (include/rtp/vtkm_compat.hpp).
#pragma once
#include <rtp/vtkm_compat.hpp>
