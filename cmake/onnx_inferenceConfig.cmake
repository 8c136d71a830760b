# Package config for the go2pi drop-in of the reference's `onnx_inference`
# package (reference: onnx_inference/CMakeLists.txt:23-33,47-53,69 exports
# onnx_inference::onnx_actor; onnx_controller/CMakeLists.txt:45-51 links it and
# the bare `onnxruntime` target). A consumer keeps
#     find_package(onnx_inference REQUIRED)
#     target_link_libraries(controller onnx_inference::onnx_actor onnxruntime ...)
# unchanged; point onnx_inference_DIR (or CMAKE_PREFIX_PATH) at this directory.
get_filename_component(_go2pi_root "${CMAKE_CURRENT_LIST_DIR}/.." ABSOLUTE)

if(NOT TARGET onnx_inference::onnx_actor)
  add_library(onnx_inference::onnx_actor SHARED IMPORTED)
  set_target_properties(onnx_inference::onnx_actor PROPERTIES
    IMPORTED_LOCATION "${_go2pi_root}/go2_onnx_controller_amd/lib/libonnx_actor.so"
    IMPORTED_SONAME "libonnx_actor.so"
    INTERFACE_INCLUDE_DIRECTORIES "${_go2pi_root}/include"
    INTERFACE_COMPILE_FEATURES cxx_std_20)
endif()

# The reference controller links the bare name `onnxruntime`; go2pi replaces
# onnxruntime entirely, so it resolves to an empty interface target.
if(NOT TARGET onnxruntime)
  add_library(onnxruntime INTERFACE IMPORTED)
endif()

set(onnx_inference_FOUND TRUE)
set(onnx_inference_VERSION 0.1)
