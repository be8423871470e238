# pdpLQRConfig.cmake -- find_package(pdpLQR) for the MI355X build.
#
# Used in place (no install step): point CMake at this directory
#   cmake -DpdpLQR_DIR=<repo>/cmake ...     (or CMAKE_PREFIX_PATH=<repo>)
# and link the imported target as with the reference package
# (README.md:52-53):  target_link_libraries(app PRIVATE pdpLQR::pdpLQR)
# The target carries the C ABI (include/pdplqr.h), the C++ facade
# (include/clqr/...) and libpdplqr.so (gfx950 code; depends on the HIP
# runtime, found through the library's RUNPATH).  Eigen3 is optional: when
# found it is linked so lqr::VectorXs / MatrixXs are Eigen types.
get_filename_component(_pdplqr_root "${CMAKE_CURRENT_LIST_DIR}/.." ABSOLUTE)
set(_pdplqr_lib "${_pdplqr_root}/pdp-lqr_amd/pdplqr/libpdplqr.so")
if(NOT EXISTS "${_pdplqr_lib}")
  set(pdpLQR_FOUND FALSE)
  set(pdpLQR_NOT_FOUND_MESSAGE
      "libpdplqr.so is not built: run make -C ${_pdplqr_root}/pdp-lqr_amd/csrc (or __graft_entry__.build())")
  return()
endif()
if(NOT TARGET pdpLQR::pdpLQR)
  add_library(pdpLQR::pdpLQR SHARED IMPORTED)
  set_target_properties(pdpLQR::pdpLQR PROPERTIES
    IMPORTED_LOCATION "${_pdplqr_lib}"
    INTERFACE_INCLUDE_DIRECTORIES "${_pdplqr_root}/include"
    INTERFACE_COMPILE_FEATURES cxx_std_17)
  find_package(Eigen3 3.3 QUIET NO_MODULE)
  if(TARGET Eigen3::Eigen)
    set_property(TARGET pdpLQR::pdpLQR APPEND PROPERTY INTERFACE_LINK_LIBRARIES Eigen3::Eigen)
  endif()
endif()
set(pdpLQR_INCLUDE_DIRS "${_pdplqr_root}/include")
set(pdpLQR_LIBRARIES pdpLQR::pdpLQR)
set(pdpLQR_FOUND TRUE)
