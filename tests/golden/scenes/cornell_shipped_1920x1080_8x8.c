#include <stdio.h>
#include <string.h>
#include <stdbool.h>
#include <math.h>
#include <unistd.h>

#include "src/libs/canvas/canvas.h"
#include "src/libs/linalg/linalg.h"
#include "src/libs/obj_loader/obj_loader.h"
#include "src/libs/photon_map/pm.h"
#include "src/color/hsl.h"
#include "src/color/lab.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"

#include "src/renderer/camera.h"
#include "src/renderer/config.h"
#include "src/renderer/photon_tracer.h"
#include "src/renderer/renderer.h"
#include "src/renderer/world.h"
#include "src/pattern/pattern.h"
#include "src/shapes/shapes.h"
#include "src/shapes/cone.h"
#include "src/shapes/csg.h"
#include "src/shapes/cube.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/group.h"
#include "src/shapes/plane.h"
#include "src/shapes/sphere.h"
#include "src/shapes/triangle.h"
#include "src/shapes/toroid.h"

#define True true
#define False false

int
main()
{
    /* config */
    struct global_config global_config;
    global_config.illumination.include_direct = True;
    global_config.illumination.include_global = False;
    global_config.illumination.debug_visualize_photon_map = False;
    global_config.illumination.debug_visualize_soft_indirect = False;
    global_config.illumination.di.include_ambient = False;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = False;
    global_config.illumination.gi.include_final_gather = True;
    global_config.illumination.gi.usteps = 8;
    global_config.illumination.gi.vsteps = 8;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/cornell_shipped_1920x1080_8x8";
    global_config.output.color_space = SRGB;

    void (*color_space_fn)(const Color, Color) = NULL;
    switch (global_config.output.color_space) {
    case RGB:
        color_space_fn = rgb_to_rgb;
        break;
    case HSL:
        color_space_fn = hsl_to_rgb;
        break;
    case XYZ:
        color_space_fn = xyz_to_rgb;
        break;
    case XYY:
        color_space_fn = xyy_to_rgb;
        break;
    case LAB:
        color_space_fn = lab_to_rgb;
        break;
    case SRGB:
        // this is the default
    default:
        color_space_fn = srgb_to_rgb;
        break;
    }

    /* end config */

    /* camera */
    struct aperture ap;
    aperture(POINT_APERTURE, 0, 8, 8, false, &ap);

    Point from = { 0.0000000000, 0.0000000000, -2.7500000000, 1.0 };
    Point to = { 0.0000000000, 0.0000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(1920, 1080, 1.2000000000/*field_of_view*/, 1.0000000000/*distance*/, 8/*usteps*/, 8/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(1);


    /* area light 0 */
    Light area_light_0 = all_lights + 0;
    Point area_light_0_corner = { 2.0000000000, 0.5000000000, 1.0000000000, 1.0};
    Color area_light_0_intensity = color(1.0000000000, 1.0000000000, 1.0000000000);
    Vector area_light_0_uvec = vector_init(0.0000000000, 1.0000000000, 0.0000000000);
    Vector area_light_0_vvec = vector_init(0.0000000000, 0.0000000000, -1.0000000000);
    area_light(area_light_0_corner, area_light_0_uvec, 10/*usteps*/, area_light_0_vvec, 10/*vsteps*/, true/*jitter*/, 65535/*cache_size*/, area_light_0_intensity, area_light_0);

    /* end area light 0 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(8);

    /* shape 0 */
    
        Pattern pattern_0_Ka = NULL;
    Pattern pattern_0_Kd = NULL;
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0 = material_alloc();
    color_space_fn(material_0_color_raw, material_0->Ka);
    color_space_fn(material_0_color_raw, material_0->Kd);
    color_space_fn(material_0_color_raw, material_0->Ks);
    color_scale(material_0->Ka, 0.1000000000);
    color_scale(material_0->Kd, 0.9000000000);
    color_scale(material_0->Ks, 0.0000000000);
    rgb_to_rgb(material_0_reflective, material_0->refl);
    rgb_to_rgb(material_0_refractive, material_0->Tf);
    material_0->reflective = material_0_reflective[0] > 0.0
                             || material_0_reflective[1] > 0.0
                             || material_0_reflective[2] > 0.0;

    material_0->Tr = 0.0000000000;
    material_0->Ns = 200.0000000000;
    material_0->Ni = 1.0000000000;
    material_0->casts_shadow = true;
    material_set_pattern(material_0, map_Ka, pattern_0_Ka);
    material_set_pattern(material_0, map_Kd, pattern_0_Kd);
    material_set_pattern(material_0, map_Ks, pattern_0_Ks);
    material_set_pattern(material_0, map_Ns, pattern_0_Ns);
    material_set_pattern(material_0, map_d, pattern_0_d);
    material_set_pattern(material_0, map_bump, pattern_0_bump);
    material_set_pattern(material_0, map_disp, pattern_0_disp);
    material_set_pattern(material_0, map_refl, pattern_0_refl);

    Matrix transform_0, transform_0_tmp;
    matrix_identity(transform_0);
    matrix_scale(1.5000000000, 0.1000000000, 1.5000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);
    matrix_translate(0.0000000000, 1.5500000000, 0.0000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);

    Shape shape_0 = all_shapes + 0;
    cube(shape_0);
    shape_set_material(shape_0, material_0);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* shape 1 */
    
        Pattern pattern_1_Ka = NULL;
    Pattern pattern_1_Kd = NULL;
    Pattern pattern_1_Ks = NULL;
    Pattern pattern_1_Ns = NULL;
    Pattern pattern_1_bump = NULL;
    Pattern pattern_1_disp = NULL;
    Pattern pattern_1_refl = NULL;
    Pattern pattern_1_d = NULL;
    Color material_1_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1 = material_alloc();
    color_space_fn(material_1_color_raw, material_1->Ka);
    color_space_fn(material_1_color_raw, material_1->Kd);
    color_space_fn(material_1_color_raw, material_1->Ks);
    color_scale(material_1->Ka, 0.1000000000);
    color_scale(material_1->Kd, 0.9000000000);
    color_scale(material_1->Ks, 0.0000000000);
    rgb_to_rgb(material_1_reflective, material_1->refl);
    rgb_to_rgb(material_1_refractive, material_1->Tf);
    material_1->reflective = material_1_reflective[0] > 0.0
                             || material_1_reflective[1] > 0.0
                             || material_1_reflective[2] > 0.0;

    material_1->Tr = 0.0000000000;
    material_1->Ns = 200.0000000000;
    material_1->Ni = 1.0000000000;
    material_1->casts_shadow = true;
    material_set_pattern(material_1, map_Ka, pattern_1_Ka);
    material_set_pattern(material_1, map_Kd, pattern_1_Kd);
    material_set_pattern(material_1, map_Ks, pattern_1_Ks);
    material_set_pattern(material_1, map_Ns, pattern_1_Ns);
    material_set_pattern(material_1, map_d, pattern_1_d);
    material_set_pattern(material_1, map_bump, pattern_1_bump);
    material_set_pattern(material_1, map_disp, pattern_1_disp);
    material_set_pattern(material_1, map_refl, pattern_1_refl);

    Matrix transform_1, transform_1_tmp;
    matrix_identity(transform_1);
    matrix_scale(1.5000000000, 0.1000000000, 1.5000000000, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);
    matrix_rotate_x(1.5707963268, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);
    matrix_translate(0.0000000000, 0.0000000000, 1.5500000000, transform_1_tmp);
    transform_chain(transform_1_tmp, transform_1);

    Shape shape_1 = all_shapes + 1;
    cube(shape_1);
    shape_set_material(shape_1, material_1);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* shape 2 */
    
        Pattern pattern_2_Ka = NULL;
    Pattern pattern_2_Kd = NULL;
    Pattern pattern_2_Ks = NULL;
    Pattern pattern_2_Ns = NULL;
    Pattern pattern_2_bump = NULL;
    Pattern pattern_2_disp = NULL;
    Pattern pattern_2_refl = NULL;
    Pattern pattern_2_d = NULL;
    Color material_2_color_raw = color(0.0100000000, 0.0100000000, 0.0100000000);
    Color material_2_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_2_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2 = material_alloc();
    color_space_fn(material_2_color_raw, material_2->Ka);
    color_space_fn(material_2_color_raw, material_2->Kd);
    color_space_fn(material_2_color_raw, material_2->Ks);
    color_scale(material_2->Ka, 0.1000000000);
    color_scale(material_2->Kd, 0.9000000000);
    color_scale(material_2->Ks, 0.0000000000);
    rgb_to_rgb(material_2_reflective, material_2->refl);
    rgb_to_rgb(material_2_refractive, material_2->Tf);
    material_2->reflective = material_2_reflective[0] > 0.0
                             || material_2_reflective[1] > 0.0
                             || material_2_reflective[2] > 0.0;

    material_2->Tr = 0.0000000000;
    material_2->Ns = 200.0000000000;
    material_2->Ni = 1.0000000000;
    material_2->casts_shadow = true;
    material_set_pattern(material_2, map_Ka, pattern_2_Ka);
    material_set_pattern(material_2, map_Kd, pattern_2_Kd);
    material_set_pattern(material_2, map_Ks, pattern_2_Ks);
    material_set_pattern(material_2, map_Ns, pattern_2_Ns);
    material_set_pattern(material_2, map_d, pattern_2_d);
    material_set_pattern(material_2, map_bump, pattern_2_bump);
    material_set_pattern(material_2, map_disp, pattern_2_disp);
    material_set_pattern(material_2, map_refl, pattern_2_refl);

    Matrix transform_2, transform_2_tmp;
    matrix_identity(transform_2);
    matrix_scale(10.0000000000, 0.0100000000, 10.0000000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_rotate_x(1.5707963268, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_translate(0.0000000000, 0.0000000000, -2.7600000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);

    Shape shape_2 = all_shapes + 2;
    cube(shape_2);
    shape_set_material(shape_2, material_2);
    shape_set_transform(shape_2, transform_2);

    /* end shape 2 */
    /* shape 3 */
    
        Pattern pattern_3_Ka = NULL;
    Pattern pattern_3_Kd = NULL;
    Pattern pattern_3_Ks = NULL;
    Pattern pattern_3_Ns = NULL;
    Pattern pattern_3_bump = NULL;
    Pattern pattern_3_disp = NULL;
    Pattern pattern_3_refl = NULL;
    Pattern pattern_3_d = NULL;
    Color material_3_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_3_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_3_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3 = material_alloc();
    color_space_fn(material_3_color_raw, material_3->Ka);
    color_space_fn(material_3_color_raw, material_3->Kd);
    color_space_fn(material_3_color_raw, material_3->Ks);
    color_scale(material_3->Ka, 0.1000000000);
    color_scale(material_3->Kd, 0.9000000000);
    color_scale(material_3->Ks, 0.0000000000);
    rgb_to_rgb(material_3_reflective, material_3->refl);
    rgb_to_rgb(material_3_refractive, material_3->Tf);
    material_3->reflective = material_3_reflective[0] > 0.0
                             || material_3_reflective[1] > 0.0
                             || material_3_reflective[2] > 0.0;

    material_3->Tr = 0.0000000000;
    material_3->Ns = 200.0000000000;
    material_3->Ni = 1.0000000000;
    material_3->casts_shadow = true;
    material_set_pattern(material_3, map_Ka, pattern_3_Ka);
    material_set_pattern(material_3, map_Kd, pattern_3_Kd);
    material_set_pattern(material_3, map_Ks, pattern_3_Ks);
    material_set_pattern(material_3, map_Ns, pattern_3_Ns);
    material_set_pattern(material_3, map_d, pattern_3_d);
    material_set_pattern(material_3, map_bump, pattern_3_bump);
    material_set_pattern(material_3, map_disp, pattern_3_disp);
    material_set_pattern(material_3, map_refl, pattern_3_refl);

    Matrix transform_3, transform_3_tmp;
    matrix_identity(transform_3);
    matrix_scale(1.5000000000, 0.1000000000, 1.5000000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);
    matrix_translate(0.0000000000, -1.5500000000, 0.0000000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);

    Shape shape_3 = all_shapes + 3;
    cube(shape_3);
    shape_set_material(shape_3, material_3);
    shape_set_transform(shape_3, transform_3);

    /* end shape 3 */
    /* shape 4 */
    
        Pattern pattern_4_Ka = NULL;
    Pattern pattern_4_Kd = NULL;
    Pattern pattern_4_Ks = NULL;
    Pattern pattern_4_Ns = NULL;
    Pattern pattern_4_bump = NULL;
    Pattern pattern_4_disp = NULL;
    Pattern pattern_4_refl = NULL;
    Pattern pattern_4_d = NULL;
    Color material_4_color_raw = color(1.0000000000, 0.0000000000, 0.0000000000);
    Color material_4_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_4_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_4 = material_alloc();
    color_space_fn(material_4_color_raw, material_4->Ka);
    color_space_fn(material_4_color_raw, material_4->Kd);
    color_space_fn(material_4_color_raw, material_4->Ks);
    color_scale(material_4->Ka, 0.1000000000);
    color_scale(material_4->Kd, 0.9000000000);
    color_scale(material_4->Ks, 0.0000000000);
    rgb_to_rgb(material_4_reflective, material_4->refl);
    rgb_to_rgb(material_4_refractive, material_4->Tf);
    material_4->reflective = material_4_reflective[0] > 0.0
                             || material_4_reflective[1] > 0.0
                             || material_4_reflective[2] > 0.0;

    material_4->Tr = 0.0000000000;
    material_4->Ns = 200.0000000000;
    material_4->Ni = 1.0000000000;
    material_4->casts_shadow = true;
    material_set_pattern(material_4, map_Ka, pattern_4_Ka);
    material_set_pattern(material_4, map_Kd, pattern_4_Kd);
    material_set_pattern(material_4, map_Ks, pattern_4_Ks);
    material_set_pattern(material_4, map_Ns, pattern_4_Ns);
    material_set_pattern(material_4, map_d, pattern_4_d);
    material_set_pattern(material_4, map_bump, pattern_4_bump);
    material_set_pattern(material_4, map_disp, pattern_4_disp);
    material_set_pattern(material_4, map_refl, pattern_4_refl);

    Matrix transform_4, transform_4_tmp;
    matrix_identity(transform_4);
    matrix_scale(1.5000000000, 0.1000000000, 1.5000000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);
    matrix_rotate_z(1.5707963268, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);
    matrix_translate(-1.5500000000, 0.0000000000, 0.0000000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);

    Shape shape_4 = all_shapes + 4;
    cube(shape_4);
    shape_set_material(shape_4, material_4);
    shape_set_transform(shape_4, transform_4);

    /* end shape 4 */
    /* shape 5 */
    
    /* children for 5 */
    Shape shape_5_children = array_of_shapes(2);
    
    /* children for 5_left */
    Shape shape_5_left_children = array_of_shapes(2);
    
        Pattern pattern_5_left_left_Ka = NULL;
    Pattern pattern_5_left_left_Kd = NULL;
    Pattern pattern_5_left_left_Ks = NULL;
    Pattern pattern_5_left_left_Ns = NULL;
    Pattern pattern_5_left_left_bump = NULL;
    Pattern pattern_5_left_left_disp = NULL;
    Pattern pattern_5_left_left_refl = NULL;
    Pattern pattern_5_left_left_d = NULL;
    Color material_5_left_left_color_raw = color(0.0000000000, 0.0000000000, 1.0000000000);
    Color material_5_left_left_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_left_left_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5_left_left = material_alloc();
    color_space_fn(material_5_left_left_color_raw, material_5_left_left->Ka);
    color_space_fn(material_5_left_left_color_raw, material_5_left_left->Kd);
    color_space_fn(material_5_left_left_color_raw, material_5_left_left->Ks);
    color_scale(material_5_left_left->Ka, 0.1000000000);
    color_scale(material_5_left_left->Kd, 0.9000000000);
    color_scale(material_5_left_left->Ks, 0.0000000000);
    rgb_to_rgb(material_5_left_left_reflective, material_5_left_left->refl);
    rgb_to_rgb(material_5_left_left_refractive, material_5_left_left->Tf);
    material_5_left_left->reflective = material_5_left_left_reflective[0] > 0.0
                             || material_5_left_left_reflective[1] > 0.0
                             || material_5_left_left_reflective[2] > 0.0;

    material_5_left_left->Tr = 0.0000000000;
    material_5_left_left->Ns = 200.0000000000;
    material_5_left_left->Ni = 1.0000000000;
    material_5_left_left->casts_shadow = true;
    material_set_pattern(material_5_left_left, map_Ka, pattern_5_left_left_Ka);
    material_set_pattern(material_5_left_left, map_Kd, pattern_5_left_left_Kd);
    material_set_pattern(material_5_left_left, map_Ks, pattern_5_left_left_Ks);
    material_set_pattern(material_5_left_left, map_Ns, pattern_5_left_left_Ns);
    material_set_pattern(material_5_left_left, map_d, pattern_5_left_left_d);
    material_set_pattern(material_5_left_left, map_bump, pattern_5_left_left_bump);
    material_set_pattern(material_5_left_left, map_disp, pattern_5_left_left_disp);
    material_set_pattern(material_5_left_left, map_refl, pattern_5_left_left_refl);

    Matrix transform_5_left_left;
    matrix_scale(1.0000000000, 0.9950000000, 1.0000000000, transform_5_left_left);
    Shape shape_5_left_left = shape_5_left_children + 0;
    cube(shape_5_left_left);
    shape_set_material(shape_5_left_left, material_5_left_left);
    shape_set_transform(shape_5_left_left, transform_5_left_left);
    
        Pattern pattern_5_left_right_Ka = NULL;
    Pattern pattern_5_left_right_Kd = NULL;
    Pattern pattern_5_left_right_Ks = NULL;
    Pattern pattern_5_left_right_Ns = NULL;
    Pattern pattern_5_left_right_bump = NULL;
    Pattern pattern_5_left_right_disp = NULL;
    Pattern pattern_5_left_right_refl = NULL;
    Pattern pattern_5_left_right_d = NULL;
    Color material_5_left_right_color_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_left_right_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_left_right_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5_left_right = material_alloc();
    color_space_fn(material_5_left_right_color_raw, material_5_left_right->Ka);
    color_space_fn(material_5_left_right_color_raw, material_5_left_right->Kd);
    color_space_fn(material_5_left_right_color_raw, material_5_left_right->Ks);
    color_scale(material_5_left_right->Ka, 0.0000000000);
    color_scale(material_5_left_right->Kd, 0.0000000000);
    color_scale(material_5_left_right->Ks, 0.0000000000);
    rgb_to_rgb(material_5_left_right_reflective, material_5_left_right->refl);
    rgb_to_rgb(material_5_left_right_refractive, material_5_left_right->Tf);
    material_5_left_right->reflective = material_5_left_right_reflective[0] > 0.0
                             || material_5_left_right_reflective[1] > 0.0
                             || material_5_left_right_reflective[2] > 0.0;

    material_5_left_right->Tr = 0.0000000000;
    material_5_left_right->Ns = 200.0000000000;
    material_5_left_right->Ni = 1.0000000000;
    material_5_left_right->casts_shadow = true;
    material_set_pattern(material_5_left_right, map_Ka, pattern_5_left_right_Ka);
    material_set_pattern(material_5_left_right, map_Kd, pattern_5_left_right_Kd);
    material_set_pattern(material_5_left_right, map_Ks, pattern_5_left_right_Ks);
    material_set_pattern(material_5_left_right, map_Ns, pattern_5_left_right_Ns);
    material_set_pattern(material_5_left_right, map_d, pattern_5_left_right_d);
    material_set_pattern(material_5_left_right, map_bump, pattern_5_left_right_bump);
    material_set_pattern(material_5_left_right, map_disp, pattern_5_left_right_disp);
    material_set_pattern(material_5_left_right, map_refl, pattern_5_left_right_refl);

    Matrix transform_5_left_right;
    matrix_translate(0.0000000000, 0.0100000000, 0.0000000000, transform_5_left_right);
    Shape shape_5_left_right = shape_5_left_children + 1;
    cube(shape_5_left_right);
    shape_set_material(shape_5_left_right, material_5_left_right);
    shape_set_transform(shape_5_left_right, transform_5_left_right);

    /* end children for 5_left */

    Matrix transform_5_left;
    matrix_identity(transform_5_left);
    Shape shape_5_left = shape_5_children + 0;
    csg(shape_5_left, CSG_UNION, shape_5_left_left, shape_5_left_right);
    shape_set_transform(shape_5_left, transform_5_left);
    
        Pattern pattern_5_right_Ka = NULL;
    Pattern pattern_5_right_Kd = NULL;
    Pattern pattern_5_right_Ks = NULL;
    Pattern pattern_5_right_Ns = NULL;
    Pattern pattern_5_right_bump = NULL;
    Pattern pattern_5_right_disp = NULL;
    Pattern pattern_5_right_refl = NULL;
    Pattern pattern_5_right_d = NULL;
    Color material_5_right_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_5_right_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_right_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5_right = material_alloc();
    color_space_fn(material_5_right_color_raw, material_5_right->Ka);
    color_space_fn(material_5_right_color_raw, material_5_right->Kd);
    color_space_fn(material_5_right_color_raw, material_5_right->Ks);
    color_scale(material_5_right->Ka, 0.1000000000);
    color_scale(material_5_right->Kd, 0.9000000000);
    color_scale(material_5_right->Ks, 0.0000000000);
    rgb_to_rgb(material_5_right_reflective, material_5_right->refl);
    rgb_to_rgb(material_5_right_refractive, material_5_right->Tf);
    material_5_right->reflective = material_5_right_reflective[0] > 0.0
                             || material_5_right_reflective[1] > 0.0
                             || material_5_right_reflective[2] > 0.0;

    material_5_right->Tr = 0.0000000000;
    material_5_right->Ns = 200.0000000000;
    material_5_right->Ni = 1.0000000000;
    material_5_right->casts_shadow = true;
    material_set_pattern(material_5_right, map_Ka, pattern_5_right_Ka);
    material_set_pattern(material_5_right, map_Kd, pattern_5_right_Kd);
    material_set_pattern(material_5_right, map_Ks, pattern_5_right_Ks);
    material_set_pattern(material_5_right, map_Ns, pattern_5_right_Ns);
    material_set_pattern(material_5_right, map_d, pattern_5_right_d);
    material_set_pattern(material_5_right, map_bump, pattern_5_right_bump);
    material_set_pattern(material_5_right, map_disp, pattern_5_right_disp);
    material_set_pattern(material_5_right, map_refl, pattern_5_right_refl);

    Matrix transform_5_right;
    matrix_scale(0.3000000000, 1.0200000000, 0.3000000000, transform_5_right);
    Shape shape_5_right = shape_5_children + 1;
    cube(shape_5_right);
    shape_set_material(shape_5_right, material_5_right);
    shape_set_transform(shape_5_right, transform_5_right);

    /* end children for 5 */

    Matrix transform_5, transform_5_tmp;
    matrix_identity(transform_5);
    matrix_scale(1.5000000000, 0.1000000000, 1.5000000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);
    matrix_rotate_z(-1.5707963268, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);
    matrix_translate(1.5500000000, 0.0000000000, 0.0000000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);

    Shape shape_5 = all_shapes + 5;
    csg(shape_5, CSG_DIFFERENCE, shape_5_left, shape_5_right);
    shape_set_transform(shape_5, transform_5);

    /* end shape 5 */
    /* shape 6 */
    
        Pattern pattern_6_Ka = NULL;
    Pattern pattern_6_Kd = NULL;
    Pattern pattern_6_Ks = NULL;
    Pattern pattern_6_Ns = NULL;
    Pattern pattern_6_bump = NULL;
    Pattern pattern_6_disp = NULL;
    Pattern pattern_6_refl = NULL;
    Pattern pattern_6_d = NULL;
    Color material_6_color_raw = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_6_reflective = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_6_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_6 = material_alloc();
    color_space_fn(material_6_color_raw, material_6->Ka);
    color_space_fn(material_6_color_raw, material_6->Kd);
    color_space_fn(material_6_color_raw, material_6->Ks);
    color_scale(material_6->Ka, 0.0000000000);
    color_scale(material_6->Kd, 0.0000000000);
    color_scale(material_6->Ks, 1.0000000000);
    rgb_to_rgb(material_6_reflective, material_6->refl);
    rgb_to_rgb(material_6_refractive, material_6->Tf);
    material_6->reflective = material_6_reflective[0] > 0.0
                             || material_6_reflective[1] > 0.0
                             || material_6_reflective[2] > 0.0;

    material_6->Tr = 0.0000000000;
    material_6->Ns = 300.0000000000;
    material_6->Ni = 1.0000000000;
    material_6->casts_shadow = true;
    material_set_pattern(material_6, map_Ka, pattern_6_Ka);
    material_set_pattern(material_6, map_Kd, pattern_6_Kd);
    material_set_pattern(material_6, map_Ks, pattern_6_Ks);
    material_set_pattern(material_6, map_Ns, pattern_6_Ns);
    material_set_pattern(material_6, map_d, pattern_6_d);
    material_set_pattern(material_6, map_bump, pattern_6_bump);
    material_set_pattern(material_6, map_disp, pattern_6_disp);
    material_set_pattern(material_6, map_refl, pattern_6_refl);

    Matrix transform_6, transform_6_tmp;
    matrix_identity(transform_6);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);
    matrix_translate(-0.6000000000, -0.7500000000, 0.5000000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);

    Shape shape_6 = all_shapes + 6;
    sphere(shape_6);
    shape_set_material(shape_6, material_6);
    shape_set_transform(shape_6, transform_6);

    /* end shape 6 */
    /* shape 7 */
    
        Pattern pattern_7_Ka = NULL;
    Pattern pattern_7_Kd = NULL;
    Pattern pattern_7_Ks = NULL;
    Pattern pattern_7_Ns = NULL;
    Pattern pattern_7_bump = NULL;
    Pattern pattern_7_disp = NULL;
    Pattern pattern_7_refl = NULL;
    Pattern pattern_7_d = NULL;
    Color material_7_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_7_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_7_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_7 = material_alloc();
    color_space_fn(material_7_color_raw, material_7->Ka);
    color_space_fn(material_7_color_raw, material_7->Kd);
    color_space_fn(material_7_color_raw, material_7->Ks);
    color_scale(material_7->Ka, 0.1000000000);
    color_scale(material_7->Kd, 0.9000000000);
    color_scale(material_7->Ks, 0.0000000000);
    rgb_to_rgb(material_7_reflective, material_7->refl);
    rgb_to_rgb(material_7_refractive, material_7->Tf);
    material_7->reflective = material_7_reflective[0] > 0.0
                             || material_7_reflective[1] > 0.0
                             || material_7_reflective[2] > 0.0;

    material_7->Tr = 0.0000000000;
    material_7->Ns = 200.0000000000;
    material_7->Ni = 1.0000000000;
    material_7->casts_shadow = true;
    material_set_pattern(material_7, map_Ka, pattern_7_Ka);
    material_set_pattern(material_7, map_Kd, pattern_7_Kd);
    material_set_pattern(material_7, map_Ks, pattern_7_Ks);
    material_set_pattern(material_7, map_Ns, pattern_7_Ns);
    material_set_pattern(material_7, map_d, pattern_7_d);
    material_set_pattern(material_7, map_bump, pattern_7_bump);
    material_set_pattern(material_7, map_disp, pattern_7_disp);
    material_set_pattern(material_7, map_refl, pattern_7_refl);

    Matrix transform_7, transform_7_tmp;
    matrix_identity(transform_7);
    matrix_scale(0.5000000000, 1.0000000000, 0.5000000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);
    matrix_translate(0.6000000000, -0.5000000000, -0.5000000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);

    Shape shape_7 = all_shapes + 7;
    cube(shape_7);
    shape_set_material(shape_7, material_7);
    shape_set_transform(shape_7, transform_7);

    /* end shape 7 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 8);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 1;
    w->shapes = world_group;
    w->shapes_num = 1;
    w->global_config = &global_config;

    if (global_config.illumination.gi.photon_count > 0 && (global_config.illumination.include_global  || global_config.illumination.debug_visualize_photon_map || global_config.illumination.debug_visualize_soft_indirect)) {
        w->photon_maps = array_of_photon_maps(3);
        printf("Tracing photons...");
        fflush(stdout);
        int i;
        for (i = 0; i < 3; ++i) {
            init_Photon_map(global_config.illumination.gi.photon_count, w->photon_maps + i);
        }
        trace_photons(w, 3, global_config.illumination.gi.include_caustics, global_config.illumination.gi.include_final_gather);
        printf("Done!\n");
        fflush(stdout);
    } else {
        w->photon_maps = NULL;
        printf("Skipping photon tracing because photon_count is 0.\n");
        fflush(stdout);
    }

    Canvas c = render_multi(cam, w, cam->usteps, cam->vsteps, cam->aperture.jitter);

    write_ppm_file(c, true, global_config.output.file_path);
    write_png(c, global_config.output.file_path);

    canvas_free(c);

    return 0;
}

