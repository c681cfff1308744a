/* frt-mi355x host API: Wavefront OBJ/MTL loader (reference src/libs/obj_loader/obj_loader.h). */
#ifndef FRT_OBJ_LOADER_H
#define FRT_OBJ_LOADER_H

#include "../../color/color.h"
#include "../../shapes/shapes.h"

void construct_group_from_obj_file(const char *file_path, void (*color_space_fn)(const Color, Color), Shape result_group);

#endif
