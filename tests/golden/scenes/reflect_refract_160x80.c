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
    global_config.illumination.di.include_ambient = True;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = False;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 1;
    global_config.illumination.gi.vsteps = 1;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/reflect_refract_160x80";
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
    aperture(POINT_APERTURE, 0, 1, 1, false, &ap);

    Point from = { -2.6000000000, 1.5000000000, -3.9000000000, 1.0 };
    Point to = { -0.6000000000, 1.0000000000, -0.8000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(160, 80, 1.1520000000/*field_of_view*/, 1.0000000000/*distance*/, 1/*usteps*/, 1/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(1);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { -4.9000000000, 4.9000000000, -1.0000000000, 1.0 };
    Color point_light_0_intensity = color(1.0000000000, 1.0000000000, 1.0000000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(13);

    /* shape 0 */
    
    Matrix transform_pattern_0_Ka;
    matrix_identity(transform_pattern_0_Ka);
    Color pattern_0_Ka_color_0_raw = color(0.3500000000, 0.3500000000, 0.3500000000);
    Color pattern_0_Ka_color_1_raw = color(0.6500000000, 0.6500000000, 0.6500000000);
    Color pattern_0_Ka_color_0;
    Color pattern_0_Ka_color_1;
    color_space_fn(pattern_0_Ka_color_0_raw, pattern_0_Ka_color_0);
    color_space_fn(pattern_0_Ka_color_1_raw, pattern_0_Ka_color_1);
    Pattern pattern_0_Ka = checker_pattern_alloc(pattern_0_Ka_color_0, pattern_0_Ka_color_1);

    pattern_set_transform(pattern_0_Ka, transform_pattern_0_Ka);
Matrix transform_pattern_0_Kd;
    matrix_identity(transform_pattern_0_Kd);
    Color pattern_0_Kd_color_0_raw = color(0.3500000000, 0.3500000000, 0.3500000000);
    Color pattern_0_Kd_color_1_raw = color(0.6500000000, 0.6500000000, 0.6500000000);
    Color pattern_0_Kd_color_0;
    Color pattern_0_Kd_color_1;
    color_space_fn(pattern_0_Kd_color_0_raw, pattern_0_Kd_color_0);
    color_space_fn(pattern_0_Kd_color_1_raw, pattern_0_Kd_color_1);
    Pattern pattern_0_Kd = checker_pattern_alloc(pattern_0_Kd_color_0, pattern_0_Kd_color_1);

    pattern_set_transform(pattern_0_Kd, transform_pattern_0_Kd);
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.4000000000, 0.4000000000, 0.4000000000);
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

    Matrix transform_0;
    matrix_rotate_y(0.3141500000, transform_0);
    Shape shape_0 = all_shapes + 0;
    plane(shape_0);
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
    Color material_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1 = material_alloc();
    color_space_fn(material_1_color_raw, material_1->Ka);
    color_space_fn(material_1_color_raw, material_1->Kd);
    color_space_fn(material_1_color_raw, material_1->Ks);
    color_scale(material_1->Ka, 0.3000000000);
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

    Matrix transform_1;
    matrix_translate(0.0000000000, 5.0000000000, 0.0000000000, transform_1);
    Shape shape_1 = all_shapes + 1;
    plane(shape_1);
    shape_set_material(shape_1, material_1);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* shape 2 */
    
    Matrix transform_pattern_2_Ka, transform_pattern_2_Ka_tmp;
    matrix_identity(transform_pattern_2_Ka);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_2_Ka_tmp);
    transform_chain(transform_pattern_2_Ka_tmp, transform_pattern_2_Ka);
    matrix_rotate_y(1.5708000000, transform_pattern_2_Ka_tmp);
    transform_chain(transform_pattern_2_Ka_tmp, transform_pattern_2_Ka);

    Color pattern_2_Ka_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_2_Ka_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_2_Ka_color_0;
    Color pattern_2_Ka_color_1;
    color_space_fn(pattern_2_Ka_color_0_raw, pattern_2_Ka_color_0);
    color_space_fn(pattern_2_Ka_color_1_raw, pattern_2_Ka_color_1);
    Pattern pattern_2_Ka = stripe_pattern_alloc(pattern_2_Ka_color_0, pattern_2_Ka_color_1);

    pattern_set_transform(pattern_2_Ka, transform_pattern_2_Ka);
Matrix transform_pattern_2_Kd, transform_pattern_2_Kd_tmp;
    matrix_identity(transform_pattern_2_Kd);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_2_Kd_tmp);
    transform_chain(transform_pattern_2_Kd_tmp, transform_pattern_2_Kd);
    matrix_rotate_y(1.5708000000, transform_pattern_2_Kd_tmp);
    transform_chain(transform_pattern_2_Kd_tmp, transform_pattern_2_Kd);

    Color pattern_2_Kd_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_2_Kd_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_2_Kd_color_0;
    Color pattern_2_Kd_color_1;
    color_space_fn(pattern_2_Kd_color_0_raw, pattern_2_Kd_color_0);
    color_space_fn(pattern_2_Kd_color_1_raw, pattern_2_Kd_color_1);
    Pattern pattern_2_Kd = stripe_pattern_alloc(pattern_2_Kd_color_0, pattern_2_Kd_color_1);

    pattern_set_transform(pattern_2_Kd, transform_pattern_2_Kd);
    Pattern pattern_2_Ks = NULL;
    Pattern pattern_2_Ns = NULL;
    Pattern pattern_2_bump = NULL;
    Pattern pattern_2_disp = NULL;
    Pattern pattern_2_refl = NULL;
    Pattern pattern_2_d = NULL;
    Color material_2_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_2_reflective = color(0.3000000000, 0.3000000000, 0.3000000000);
    Color material_2_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2 = material_alloc();
    color_space_fn(material_2_color_raw, material_2->Ka);
    color_space_fn(material_2_color_raw, material_2->Kd);
    color_space_fn(material_2_color_raw, material_2->Ks);
    color_scale(material_2->Ka, 0.0000000000);
    color_scale(material_2->Kd, 0.4000000000);
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
    matrix_rotate_y(1.5708000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_rotate_z(1.5708000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);
    matrix_translate(-5.0000000000, 0.0000000000, 0.0000000000, transform_2_tmp);
    transform_chain(transform_2_tmp, transform_2);

    Shape shape_2 = all_shapes + 2;
    plane(shape_2);
    shape_set_material(shape_2, material_2);
    shape_set_transform(shape_2, transform_2);

    /* end shape 2 */
    /* shape 3 */
    
    Matrix transform_pattern_3_Ka, transform_pattern_3_Ka_tmp;
    matrix_identity(transform_pattern_3_Ka);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_3_Ka_tmp);
    transform_chain(transform_pattern_3_Ka_tmp, transform_pattern_3_Ka);
    matrix_rotate_y(1.5708000000, transform_pattern_3_Ka_tmp);
    transform_chain(transform_pattern_3_Ka_tmp, transform_pattern_3_Ka);

    Color pattern_3_Ka_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_3_Ka_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_3_Ka_color_0;
    Color pattern_3_Ka_color_1;
    color_space_fn(pattern_3_Ka_color_0_raw, pattern_3_Ka_color_0);
    color_space_fn(pattern_3_Ka_color_1_raw, pattern_3_Ka_color_1);
    Pattern pattern_3_Ka = stripe_pattern_alloc(pattern_3_Ka_color_0, pattern_3_Ka_color_1);

    pattern_set_transform(pattern_3_Ka, transform_pattern_3_Ka);
Matrix transform_pattern_3_Kd, transform_pattern_3_Kd_tmp;
    matrix_identity(transform_pattern_3_Kd);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_3_Kd_tmp);
    transform_chain(transform_pattern_3_Kd_tmp, transform_pattern_3_Kd);
    matrix_rotate_y(1.5708000000, transform_pattern_3_Kd_tmp);
    transform_chain(transform_pattern_3_Kd_tmp, transform_pattern_3_Kd);

    Color pattern_3_Kd_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_3_Kd_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_3_Kd_color_0;
    Color pattern_3_Kd_color_1;
    color_space_fn(pattern_3_Kd_color_0_raw, pattern_3_Kd_color_0);
    color_space_fn(pattern_3_Kd_color_1_raw, pattern_3_Kd_color_1);
    Pattern pattern_3_Kd = stripe_pattern_alloc(pattern_3_Kd_color_0, pattern_3_Kd_color_1);

    pattern_set_transform(pattern_3_Kd, transform_pattern_3_Kd);
    Pattern pattern_3_Ks = NULL;
    Pattern pattern_3_Ns = NULL;
    Pattern pattern_3_bump = NULL;
    Pattern pattern_3_disp = NULL;
    Pattern pattern_3_refl = NULL;
    Pattern pattern_3_d = NULL;
    Color material_3_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_3_reflective = color(0.3000000000, 0.3000000000, 0.3000000000);
    Color material_3_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3 = material_alloc();
    color_space_fn(material_3_color_raw, material_3->Ka);
    color_space_fn(material_3_color_raw, material_3->Kd);
    color_space_fn(material_3_color_raw, material_3->Ks);
    color_scale(material_3->Ka, 0.0000000000);
    color_scale(material_3->Kd, 0.4000000000);
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
    matrix_rotate_y(1.5708000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);
    matrix_rotate_z(1.5708000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);
    matrix_translate(5.0000000000, 0.0000000000, 0.0000000000, transform_3_tmp);
    transform_chain(transform_3_tmp, transform_3);

    Shape shape_3 = all_shapes + 3;
    plane(shape_3);
    shape_set_material(shape_3, material_3);
    shape_set_transform(shape_3, transform_3);

    /* end shape 3 */
    /* shape 4 */
    
    Matrix transform_pattern_4_Ka, transform_pattern_4_Ka_tmp;
    matrix_identity(transform_pattern_4_Ka);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_4_Ka_tmp);
    transform_chain(transform_pattern_4_Ka_tmp, transform_pattern_4_Ka);
    matrix_rotate_y(1.5708000000, transform_pattern_4_Ka_tmp);
    transform_chain(transform_pattern_4_Ka_tmp, transform_pattern_4_Ka);

    Color pattern_4_Ka_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_4_Ka_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_4_Ka_color_0;
    Color pattern_4_Ka_color_1;
    color_space_fn(pattern_4_Ka_color_0_raw, pattern_4_Ka_color_0);
    color_space_fn(pattern_4_Ka_color_1_raw, pattern_4_Ka_color_1);
    Pattern pattern_4_Ka = stripe_pattern_alloc(pattern_4_Ka_color_0, pattern_4_Ka_color_1);

    pattern_set_transform(pattern_4_Ka, transform_pattern_4_Ka);
Matrix transform_pattern_4_Kd, transform_pattern_4_Kd_tmp;
    matrix_identity(transform_pattern_4_Kd);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_4_Kd_tmp);
    transform_chain(transform_pattern_4_Kd_tmp, transform_pattern_4_Kd);
    matrix_rotate_y(1.5708000000, transform_pattern_4_Kd_tmp);
    transform_chain(transform_pattern_4_Kd_tmp, transform_pattern_4_Kd);

    Color pattern_4_Kd_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_4_Kd_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_4_Kd_color_0;
    Color pattern_4_Kd_color_1;
    color_space_fn(pattern_4_Kd_color_0_raw, pattern_4_Kd_color_0);
    color_space_fn(pattern_4_Kd_color_1_raw, pattern_4_Kd_color_1);
    Pattern pattern_4_Kd = stripe_pattern_alloc(pattern_4_Kd_color_0, pattern_4_Kd_color_1);

    pattern_set_transform(pattern_4_Kd, transform_pattern_4_Kd);
    Pattern pattern_4_Ks = NULL;
    Pattern pattern_4_Ns = NULL;
    Pattern pattern_4_bump = NULL;
    Pattern pattern_4_disp = NULL;
    Pattern pattern_4_refl = NULL;
    Pattern pattern_4_d = NULL;
    Color material_4_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_4_reflective = color(0.3000000000, 0.3000000000, 0.3000000000);
    Color material_4_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_4 = material_alloc();
    color_space_fn(material_4_color_raw, material_4->Ka);
    color_space_fn(material_4_color_raw, material_4->Kd);
    color_space_fn(material_4_color_raw, material_4->Ks);
    color_scale(material_4->Ka, 0.0000000000);
    color_scale(material_4->Kd, 0.4000000000);
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
    matrix_rotate_x(1.5708000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);
    matrix_translate(0.0000000000, 0.0000000000, 5.0000000000, transform_4_tmp);
    transform_chain(transform_4_tmp, transform_4);

    Shape shape_4 = all_shapes + 4;
    plane(shape_4);
    shape_set_material(shape_4, material_4);
    shape_set_transform(shape_4, transform_4);

    /* end shape 4 */
    /* shape 5 */
    
    Matrix transform_pattern_5_Ka, transform_pattern_5_Ka_tmp;
    matrix_identity(transform_pattern_5_Ka);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_5_Ka_tmp);
    transform_chain(transform_pattern_5_Ka_tmp, transform_pattern_5_Ka);
    matrix_rotate_y(1.5708000000, transform_pattern_5_Ka_tmp);
    transform_chain(transform_pattern_5_Ka_tmp, transform_pattern_5_Ka);

    Color pattern_5_Ka_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_5_Ka_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_5_Ka_color_0;
    Color pattern_5_Ka_color_1;
    color_space_fn(pattern_5_Ka_color_0_raw, pattern_5_Ka_color_0);
    color_space_fn(pattern_5_Ka_color_1_raw, pattern_5_Ka_color_1);
    Pattern pattern_5_Ka = stripe_pattern_alloc(pattern_5_Ka_color_0, pattern_5_Ka_color_1);

    pattern_set_transform(pattern_5_Ka, transform_pattern_5_Ka);
Matrix transform_pattern_5_Kd, transform_pattern_5_Kd_tmp;
    matrix_identity(transform_pattern_5_Kd);
    matrix_scale(0.2500000000, 0.2500000000, 0.2500000000, transform_pattern_5_Kd_tmp);
    transform_chain(transform_pattern_5_Kd_tmp, transform_pattern_5_Kd);
    matrix_rotate_y(1.5708000000, transform_pattern_5_Kd_tmp);
    transform_chain(transform_pattern_5_Kd_tmp, transform_pattern_5_Kd);

    Color pattern_5_Kd_color_0_raw = color(0.4500000000, 0.4500000000, 0.4500000000);
    Color pattern_5_Kd_color_1_raw = color(0.5500000000, 0.5500000000, 0.5500000000);
    Color pattern_5_Kd_color_0;
    Color pattern_5_Kd_color_1;
    color_space_fn(pattern_5_Kd_color_0_raw, pattern_5_Kd_color_0);
    color_space_fn(pattern_5_Kd_color_1_raw, pattern_5_Kd_color_1);
    Pattern pattern_5_Kd = stripe_pattern_alloc(pattern_5_Kd_color_0, pattern_5_Kd_color_1);

    pattern_set_transform(pattern_5_Kd, transform_pattern_5_Kd);
    Pattern pattern_5_Ks = NULL;
    Pattern pattern_5_Ns = NULL;
    Pattern pattern_5_bump = NULL;
    Pattern pattern_5_disp = NULL;
    Pattern pattern_5_refl = NULL;
    Pattern pattern_5_d = NULL;
    Color material_5_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_5_reflective = color(0.3000000000, 0.3000000000, 0.3000000000);
    Color material_5_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5 = material_alloc();
    color_space_fn(material_5_color_raw, material_5->Ka);
    color_space_fn(material_5_color_raw, material_5->Kd);
    color_space_fn(material_5_color_raw, material_5->Ks);
    color_scale(material_5->Ka, 0.0000000000);
    color_scale(material_5->Kd, 0.4000000000);
    color_scale(material_5->Ks, 0.0000000000);
    rgb_to_rgb(material_5_reflective, material_5->refl);
    rgb_to_rgb(material_5_refractive, material_5->Tf);
    material_5->reflective = material_5_reflective[0] > 0.0
                             || material_5_reflective[1] > 0.0
                             || material_5_reflective[2] > 0.0;

    material_5->Tr = 0.0000000000;
    material_5->Ns = 200.0000000000;
    material_5->Ni = 1.0000000000;
    material_5->casts_shadow = true;
    material_set_pattern(material_5, map_Ka, pattern_5_Ka);
    material_set_pattern(material_5, map_Kd, pattern_5_Kd);
    material_set_pattern(material_5, map_Ks, pattern_5_Ks);
    material_set_pattern(material_5, map_Ns, pattern_5_Ns);
    material_set_pattern(material_5, map_d, pattern_5_d);
    material_set_pattern(material_5, map_bump, pattern_5_bump);
    material_set_pattern(material_5, map_disp, pattern_5_disp);
    material_set_pattern(material_5, map_refl, pattern_5_refl);

    Matrix transform_5, transform_5_tmp;
    matrix_identity(transform_5);
    matrix_rotate_x(1.5708000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);
    matrix_translate(0.0000000000, 0.0000000000, -5.0000000000, transform_5_tmp);
    transform_chain(transform_5_tmp, transform_5);

    Shape shape_5 = all_shapes + 5;
    plane(shape_5);
    shape_set_material(shape_5, material_5);
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
    Color material_6_color_raw = color(0.8000000000, 0.5000000000, 0.3000000000);
    Color material_6_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_6_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_6 = material_alloc();
    color_space_fn(material_6_color_raw, material_6->Ka);
    color_space_fn(material_6_color_raw, material_6->Kd);
    color_space_fn(material_6_color_raw, material_6->Ks);
    color_scale(material_6->Ka, 0.1000000000);
    color_scale(material_6->Kd, 0.9000000000);
    color_scale(material_6->Ks, 0.9000000000);
    rgb_to_rgb(material_6_reflective, material_6->refl);
    rgb_to_rgb(material_6_refractive, material_6->Tf);
    material_6->reflective = material_6_reflective[0] > 0.0
                             || material_6_reflective[1] > 0.0
                             || material_6_reflective[2] > 0.0;

    material_6->Tr = 0.0000000000;
    material_6->Ns = 50.0000000000;
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
    matrix_scale(0.4000000000, 0.4000000000, 0.4000000000, transform_6_tmp);
    transform_chain(transform_6_tmp, transform_6);
    matrix_translate(4.6000000000, 0.4000000000, 1.0000000000, transform_6_tmp);
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
    Color material_7_color_raw = color(0.9000000000, 0.4000000000, 0.5000000000);
    Color material_7_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_7_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_7 = material_alloc();
    color_space_fn(material_7_color_raw, material_7->Ka);
    color_space_fn(material_7_color_raw, material_7->Kd);
    color_space_fn(material_7_color_raw, material_7->Ks);
    color_scale(material_7->Ka, 0.1000000000);
    color_scale(material_7->Kd, 0.9000000000);
    color_scale(material_7->Ks, 0.9000000000);
    rgb_to_rgb(material_7_reflective, material_7->refl);
    rgb_to_rgb(material_7_refractive, material_7->Tf);
    material_7->reflective = material_7_reflective[0] > 0.0
                             || material_7_reflective[1] > 0.0
                             || material_7_reflective[2] > 0.0;

    material_7->Tr = 0.0000000000;
    material_7->Ns = 50.0000000000;
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
    matrix_scale(0.3000000000, 0.3000000000, 0.3000000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);
    matrix_translate(4.7000000000, 0.3000000000, 0.4000000000, transform_7_tmp);
    transform_chain(transform_7_tmp, transform_7);

    Shape shape_7 = all_shapes + 7;
    sphere(shape_7);
    shape_set_material(shape_7, material_7);
    shape_set_transform(shape_7, transform_7);

    /* end shape 7 */
    /* shape 8 */
    
        Pattern pattern_8_Ka = NULL;
    Pattern pattern_8_Kd = NULL;
    Pattern pattern_8_Ks = NULL;
    Pattern pattern_8_Ns = NULL;
    Pattern pattern_8_bump = NULL;
    Pattern pattern_8_disp = NULL;
    Pattern pattern_8_refl = NULL;
    Pattern pattern_8_d = NULL;
    Color material_8_color_raw = color(0.4000000000, 0.9000000000, 0.6000000000);
    Color material_8_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_8_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_8 = material_alloc();
    color_space_fn(material_8_color_raw, material_8->Ka);
    color_space_fn(material_8_color_raw, material_8->Kd);
    color_space_fn(material_8_color_raw, material_8->Ks);
    color_scale(material_8->Ka, 0.1000000000);
    color_scale(material_8->Kd, 0.9000000000);
    color_scale(material_8->Ks, 0.9000000000);
    rgb_to_rgb(material_8_reflective, material_8->refl);
    rgb_to_rgb(material_8_refractive, material_8->Tf);
    material_8->reflective = material_8_reflective[0] > 0.0
                             || material_8_reflective[1] > 0.0
                             || material_8_reflective[2] > 0.0;

    material_8->Tr = 0.0000000000;
    material_8->Ns = 50.0000000000;
    material_8->Ni = 1.0000000000;
    material_8->casts_shadow = true;
    material_set_pattern(material_8, map_Ka, pattern_8_Ka);
    material_set_pattern(material_8, map_Kd, pattern_8_Kd);
    material_set_pattern(material_8, map_Ks, pattern_8_Ks);
    material_set_pattern(material_8, map_Ns, pattern_8_Ns);
    material_set_pattern(material_8, map_d, pattern_8_d);
    material_set_pattern(material_8, map_bump, pattern_8_bump);
    material_set_pattern(material_8, map_disp, pattern_8_disp);
    material_set_pattern(material_8, map_refl, pattern_8_refl);

    Matrix transform_8, transform_8_tmp;
    matrix_identity(transform_8);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_8_tmp);
    transform_chain(transform_8_tmp, transform_8);
    matrix_translate(-1.0000000000, 0.5000000000, 4.5000000000, transform_8_tmp);
    transform_chain(transform_8_tmp, transform_8);

    Shape shape_8 = all_shapes + 8;
    sphere(shape_8);
    shape_set_material(shape_8, material_8);
    shape_set_transform(shape_8, transform_8);

    /* end shape 8 */
    /* shape 9 */
    
        Pattern pattern_9_Ka = NULL;
    Pattern pattern_9_Kd = NULL;
    Pattern pattern_9_Ks = NULL;
    Pattern pattern_9_Ns = NULL;
    Pattern pattern_9_bump = NULL;
    Pattern pattern_9_disp = NULL;
    Pattern pattern_9_refl = NULL;
    Pattern pattern_9_d = NULL;
    Color material_9_color_raw = color(0.4000000000, 0.6000000000, 0.9000000000);
    Color material_9_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_9_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_9 = material_alloc();
    color_space_fn(material_9_color_raw, material_9->Ka);
    color_space_fn(material_9_color_raw, material_9->Kd);
    color_space_fn(material_9_color_raw, material_9->Ks);
    color_scale(material_9->Ka, 0.1000000000);
    color_scale(material_9->Kd, 0.9000000000);
    color_scale(material_9->Ks, 0.9000000000);
    rgb_to_rgb(material_9_reflective, material_9->refl);
    rgb_to_rgb(material_9_refractive, material_9->Tf);
    material_9->reflective = material_9_reflective[0] > 0.0
                             || material_9_reflective[1] > 0.0
                             || material_9_reflective[2] > 0.0;

    material_9->Tr = 0.0000000000;
    material_9->Ns = 50.0000000000;
    material_9->Ni = 1.0000000000;
    material_9->casts_shadow = true;
    material_set_pattern(material_9, map_Ka, pattern_9_Ka);
    material_set_pattern(material_9, map_Kd, pattern_9_Kd);
    material_set_pattern(material_9, map_Ks, pattern_9_Ks);
    material_set_pattern(material_9, map_Ns, pattern_9_Ns);
    material_set_pattern(material_9, map_d, pattern_9_d);
    material_set_pattern(material_9, map_bump, pattern_9_bump);
    material_set_pattern(material_9, map_disp, pattern_9_disp);
    material_set_pattern(material_9, map_refl, pattern_9_refl);

    Matrix transform_9, transform_9_tmp;
    matrix_identity(transform_9);
    matrix_scale(0.3000000000, 0.3000000000, 0.3000000000, transform_9_tmp);
    transform_chain(transform_9_tmp, transform_9);
    matrix_translate(-1.7000000000, 0.3000000000, 4.7000000000, transform_9_tmp);
    transform_chain(transform_9_tmp, transform_9);

    Shape shape_9 = all_shapes + 9;
    sphere(shape_9);
    shape_set_material(shape_9, material_9);
    shape_set_transform(shape_9, transform_9);

    /* end shape 9 */
    /* shape 10 */
    
        Pattern pattern_10_Ka = NULL;
    Pattern pattern_10_Kd = NULL;
    Pattern pattern_10_Ks = NULL;
    Pattern pattern_10_Ns = NULL;
    Pattern pattern_10_bump = NULL;
    Pattern pattern_10_disp = NULL;
    Pattern pattern_10_refl = NULL;
    Pattern pattern_10_d = NULL;
    Color material_10_color_raw = color(1.0000000000, 0.3000000000, 0.2000000000);
    Color material_10_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_10_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_10 = material_alloc();
    color_space_fn(material_10_color_raw, material_10->Ka);
    color_space_fn(material_10_color_raw, material_10->Kd);
    color_space_fn(material_10_color_raw, material_10->Ks);
    color_scale(material_10->Ka, 0.1000000000);
    color_scale(material_10->Kd, 0.9000000000);
    color_scale(material_10->Ks, 0.4000000000);
    rgb_to_rgb(material_10_reflective, material_10->refl);
    rgb_to_rgb(material_10_refractive, material_10->Tf);
    material_10->reflective = material_10_reflective[0] > 0.0
                             || material_10_reflective[1] > 0.0
                             || material_10_reflective[2] > 0.0;

    material_10->Tr = 0.0000000000;
    material_10->Ns = 5.0000000000;
    material_10->Ni = 1.0000000000;
    material_10->casts_shadow = true;
    material_set_pattern(material_10, map_Ka, pattern_10_Ka);
    material_set_pattern(material_10, map_Kd, pattern_10_Kd);
    material_set_pattern(material_10, map_Ks, pattern_10_Ks);
    material_set_pattern(material_10, map_Ns, pattern_10_Ns);
    material_set_pattern(material_10, map_d, pattern_10_d);
    material_set_pattern(material_10, map_bump, pattern_10_bump);
    material_set_pattern(material_10, map_disp, pattern_10_disp);
    material_set_pattern(material_10, map_refl, pattern_10_refl);

    Matrix transform_10;
    matrix_translate(-0.6000000000, 1.0000000000, 0.6000000000, transform_10);
    Shape shape_10 = all_shapes + 10;
    sphere(shape_10);
    shape_set_material(shape_10, material_10);
    shape_set_transform(shape_10, transform_10);

    /* end shape 10 */
    /* shape 11 */
    
        Pattern pattern_11_Ka = NULL;
    Pattern pattern_11_Kd = NULL;
    Pattern pattern_11_Ks = NULL;
    Pattern pattern_11_Ns = NULL;
    Pattern pattern_11_bump = NULL;
    Pattern pattern_11_disp = NULL;
    Pattern pattern_11_refl = NULL;
    Pattern pattern_11_d = NULL;
    Color material_11_color_raw = color(0.0000000000, 0.0000000000, 0.2000000000);
    Color material_11_reflective = color(0.9000000000, 0.9000000000, 0.9000000000);
    Color material_11_refractive = color(0.9000000000, 0.9000000000, 0.9000000000);

    Material material_11 = material_alloc();
    color_space_fn(material_11_color_raw, material_11->Ka);
    color_space_fn(material_11_color_raw, material_11->Kd);
    color_space_fn(material_11_color_raw, material_11->Ks);
    color_scale(material_11->Ka, 0.0000000000);
    color_scale(material_11->Kd, 0.4000000000);
    color_scale(material_11->Ks, 0.9000000000);
    rgb_to_rgb(material_11_reflective, material_11->refl);
    rgb_to_rgb(material_11_refractive, material_11->Tf);
    material_11->reflective = material_11_reflective[0] > 0.0
                             || material_11_reflective[1] > 0.0
                             || material_11_reflective[2] > 0.0;

    material_11->Tr = 0.9000000000;
    material_11->Ns = 300.0000000000;
    material_11->Ni = 1.5000000000;
    material_11->casts_shadow = true;
    material_set_pattern(material_11, map_Ka, pattern_11_Ka);
    material_set_pattern(material_11, map_Kd, pattern_11_Kd);
    material_set_pattern(material_11, map_Ks, pattern_11_Ks);
    material_set_pattern(material_11, map_Ns, pattern_11_Ns);
    material_set_pattern(material_11, map_d, pattern_11_d);
    material_set_pattern(material_11, map_bump, pattern_11_bump);
    material_set_pattern(material_11, map_disp, pattern_11_disp);
    material_set_pattern(material_11, map_refl, pattern_11_refl);

    Matrix transform_11, transform_11_tmp;
    matrix_identity(transform_11);
    matrix_scale(0.7000000000, 0.7000000000, 0.7000000000, transform_11_tmp);
    transform_chain(transform_11_tmp, transform_11);
    matrix_translate(0.6000000000, 0.7000000000, -0.6000000000, transform_11_tmp);
    transform_chain(transform_11_tmp, transform_11);

    Shape shape_11 = all_shapes + 11;
    sphere(shape_11);
    shape_set_material(shape_11, material_11);
    shape_set_transform(shape_11, transform_11);

    /* end shape 11 */
    /* shape 12 */
    
        Pattern pattern_12_Ka = NULL;
    Pattern pattern_12_Kd = NULL;
    Pattern pattern_12_Ks = NULL;
    Pattern pattern_12_Ns = NULL;
    Pattern pattern_12_bump = NULL;
    Pattern pattern_12_disp = NULL;
    Pattern pattern_12_refl = NULL;
    Pattern pattern_12_d = NULL;
    Color material_12_color_raw = color(0.0000000000, 0.2000000000, 0.0000000000);
    Color material_12_reflective = color(0.9000000000, 0.9000000000, 0.9000000000);
    Color material_12_refractive = color(0.9000000000, 0.9000000000, 0.9000000000);

    Material material_12 = material_alloc();
    color_space_fn(material_12_color_raw, material_12->Ka);
    color_space_fn(material_12_color_raw, material_12->Kd);
    color_space_fn(material_12_color_raw, material_12->Ks);
    color_scale(material_12->Ka, 0.0000000000);
    color_scale(material_12->Kd, 0.4000000000);
    color_scale(material_12->Ks, 0.9000000000);
    rgb_to_rgb(material_12_reflective, material_12->refl);
    rgb_to_rgb(material_12_refractive, material_12->Tf);
    material_12->reflective = material_12_reflective[0] > 0.0
                             || material_12_reflective[1] > 0.0
                             || material_12_reflective[2] > 0.0;

    material_12->Tr = 0.9000000000;
    material_12->Ns = 300.0000000000;
    material_12->Ni = 1.5000000000;
    material_12->casts_shadow = true;
    material_set_pattern(material_12, map_Ka, pattern_12_Ka);
    material_set_pattern(material_12, map_Kd, pattern_12_Kd);
    material_set_pattern(material_12, map_Ks, pattern_12_Ks);
    material_set_pattern(material_12, map_Ns, pattern_12_Ns);
    material_set_pattern(material_12, map_d, pattern_12_d);
    material_set_pattern(material_12, map_bump, pattern_12_bump);
    material_set_pattern(material_12, map_disp, pattern_12_disp);
    material_set_pattern(material_12, map_refl, pattern_12_refl);

    Matrix transform_12, transform_12_tmp;
    matrix_identity(transform_12);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_12_tmp);
    transform_chain(transform_12_tmp, transform_12);
    matrix_translate(-0.7000000000, 0.5000000000, -0.8000000000, transform_12_tmp);
    transform_chain(transform_12_tmp, transform_12);

    Shape shape_12 = all_shapes + 12;
    sphere(shape_12);
    shape_set_material(shape_12, material_12);
    shape_set_transform(shape_12, transform_12);

    /* end shape 12 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 13);
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

