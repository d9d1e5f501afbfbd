// lib.hip — single translation unit for the device code + the C-ABI (kernels are launched
// from the same TU that defines them; no relocatable device code needed).
#include "kernels.hip"
#include "vanish.hip"
#include "json_pack.hip"
#include "api.cpp"
