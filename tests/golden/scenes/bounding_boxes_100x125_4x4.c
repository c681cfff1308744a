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

    global_config.illumination.gi.include_caustics = True;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 8;
    global_config.illumination.gi.vsteps = 8;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/bounding_boxes_100x125_4x4";
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
    aperture(POINT_APERTURE, 0, 4, 4, false, &ap);

    Point from = { 0.0000000000, 2.5000000000, -10.0000000000, 1.0 };
    Point to = { 0.0000000000, 1.0000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(100, 125, 1.2000000000/*field_of_view*/, 1.0000000000/*distance*/, 4/*usteps*/, 4/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(4);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { -10.0000000000, 100.0000000000, -100.0000000000, 1.0 };
    Color point_light_0_intensity = color(1.6000000000, 1.6000000000, 1.6000000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */
    /* point light 1 */
    Light point_light_1 = all_lights + 1;
    Point point_light_1_point = { 0.0000000000, 100.0000000000, 0.0000000000, 1.0 };
    Color point_light_1_intensity = color(0.4000000000, 0.4000000000, 0.4000000000);
    point_light(point_light_1_point, point_light_1_intensity, point_light_1);

    /* end point light 1 */
    /* point light 2 */
    Light point_light_2 = all_lights + 2;
    Point point_light_2_point = { 100.0000000000, 10.0000000000, -25.0000000000, 1.0 };
    Color point_light_2_intensity = color(0.8000000000, 0.8000000000, 0.8000000000);
    point_light(point_light_2_point, point_light_2_intensity, point_light_2);

    /* end point light 2 */
    /* point light 3 */
    Light point_light_3 = all_lights + 3;
    Point point_light_3_point = { -100.0000000000, 10.0000000000, -25.0000000000, 1.0 };
    Color point_light_3_intensity = color(0.8000000000, 0.8000000000, 0.8000000000);
    point_light(point_light_3_point, point_light_3_intensity, point_light_3);

    /* end point light 3 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(6);

    /* shape 0 */
    
    /* children for 0 */
    Shape shape_0_children = array_of_shapes(2);

    
        Pattern pattern_0_child_0_Ka = NULL;
    Pattern pattern_0_child_0_Kd = NULL;
    Pattern pattern_0_child_0_Ks = NULL;
    Pattern pattern_0_child_0_Ns = NULL;
    Pattern pattern_0_child_0_bump = NULL;
    Pattern pattern_0_child_0_disp = NULL;
    Pattern pattern_0_child_0_refl = NULL;
    Pattern pattern_0_child_0_d = NULL;
    Color material_0_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_0_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_0_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0_child_0 = material_alloc();
    color_space_fn(material_0_child_0_color_raw, material_0_child_0->Ka);
    color_space_fn(material_0_child_0_color_raw, material_0_child_0->Kd);
    color_space_fn(material_0_child_0_color_raw, material_0_child_0->Ks);
    color_scale(material_0_child_0->Ka, 0.0000000000);
    color_scale(material_0_child_0->Kd, 0.8000000000);
    color_scale(material_0_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_0_child_0_reflective, material_0_child_0->refl);
    rgb_to_rgb(material_0_child_0_refractive, material_0_child_0->Tf);
    material_0_child_0->reflective = material_0_child_0_reflective[0] > 0.0
                             || material_0_child_0_reflective[1] > 0.0
                             || material_0_child_0_reflective[2] > 0.0;

    material_0_child_0->Tr = 0.0000000000;
    material_0_child_0->Ns = 200.0000000000;
    material_0_child_0->Ni = 1.0000000000;
    material_0_child_0->casts_shadow = true;
    material_set_pattern(material_0_child_0, map_Ka, pattern_0_child_0_Ka);
    material_set_pattern(material_0_child_0, map_Kd, pattern_0_child_0_Kd);
    material_set_pattern(material_0_child_0, map_Ks, pattern_0_child_0_Ks);
    material_set_pattern(material_0_child_0, map_Ns, pattern_0_child_0_Ns);
    material_set_pattern(material_0_child_0, map_d, pattern_0_child_0_d);
    material_set_pattern(material_0_child_0, map_bump, pattern_0_child_0_bump);
    material_set_pattern(material_0_child_0, map_disp, pattern_0_child_0_disp);
    material_set_pattern(material_0_child_0, map_refl, pattern_0_child_0_refl);

    Matrix transform_0_child_0;
    matrix_identity(transform_0_child_0);
    Shape shape_0_child_0 = shape_0_children + 0;
    cylinder(shape_0_child_0);
    shape_set_material(shape_0_child_0, material_0_child_0);
    shape_set_transform(shape_0_child_0, transform_0_child_0);
    shape_0_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_0_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_0_child_0->fields.cylinder.closed = true;


    
    /* children for 0_child_1 */
    Shape shape_0_child_1_children = array_of_shapes(2);

        Pattern pattern_0_child_1_child_0_Ka = NULL;
    Pattern pattern_0_child_1_child_0_Kd = NULL;
    Pattern pattern_0_child_1_child_0_Ks = NULL;
    Pattern pattern_0_child_1_child_0_Ns = NULL;
    Pattern pattern_0_child_1_child_0_bump = NULL;
    Pattern pattern_0_child_1_child_0_disp = NULL;
    Pattern pattern_0_child_1_child_0_refl = NULL;
    Pattern pattern_0_child_1_child_0_d = NULL;
    Color material_0_child_1_child_0_color_raw = color(1.0000000000, 0.0000000000, 0.1000000000);
    Color material_0_child_1_child_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_child_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0_child_1_child_0 = material_alloc();
    color_space_fn(material_0_child_1_child_0_color_raw, material_0_child_1_child_0->Ka);
    color_space_fn(material_0_child_1_child_0_color_raw, material_0_child_1_child_0->Kd);
    color_space_fn(material_0_child_1_child_0_color_raw, material_0_child_1_child_0->Ks);
    color_scale(material_0_child_1_child_0->Ka, 0.1000000000);
    color_scale(material_0_child_1_child_0->Kd, 0.6000000000);
    color_scale(material_0_child_1_child_0->Ks, 0.8000000000);
    rgb_to_rgb(material_0_child_1_child_0_reflective, material_0_child_1_child_0->refl);
    rgb_to_rgb(material_0_child_1_child_0_refractive, material_0_child_1_child_0->Tf);
    material_0_child_1_child_0->reflective = material_0_child_1_child_0_reflective[0] > 0.0
                             || material_0_child_1_child_0_reflective[1] > 0.0
                             || material_0_child_1_child_0_reflective[2] > 0.0;

    material_0_child_1_child_0->Tr = 0.0000000000;
    material_0_child_1_child_0->Ns = 15.0000000000;
    material_0_child_1_child_0->Ni = 1.0000000000;
    material_0_child_1_child_0->casts_shadow = true;
    material_set_pattern(material_0_child_1_child_0, map_Ka, pattern_0_child_1_child_0_Ka);
    material_set_pattern(material_0_child_1_child_0, map_Kd, pattern_0_child_1_child_0_Kd);
    material_set_pattern(material_0_child_1_child_0, map_Ks, pattern_0_child_1_child_0_Ks);
    material_set_pattern(material_0_child_1_child_0, map_Ns, pattern_0_child_1_child_0_Ns);
    material_set_pattern(material_0_child_1_child_0, map_d, pattern_0_child_1_child_0_d);
    material_set_pattern(material_0_child_1_child_0, map_bump, pattern_0_child_1_child_0_bump);
    material_set_pattern(material_0_child_1_child_0, map_disp, pattern_0_child_1_child_0_disp);
    material_set_pattern(material_0_child_1_child_0, map_refl, pattern_0_child_1_child_0_refl);

    Matrix transform_0_child_1_child_0, transform_0_child_1_child_0_tmp;
    matrix_identity(transform_0_child_1_child_0);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_0_child_1_child_0_tmp);
    transform_chain(transform_0_child_1_child_0_tmp, transform_0_child_1_child_0);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_0_child_1_child_0_tmp);
    transform_chain(transform_0_child_1_child_0_tmp, transform_0_child_1_child_0);

    Shape shape_0_child_1_child_0 = shape_0_child_1_children + 0;

    if (access("scenes/bounding_boxes/dragon.obj", F_OK ) == -1 ) {
        printf("file 'scenes/bounding_boxes/dragon.obj' does not exist.");
        return 1;
    }
    printf("Loading resource 'scenes/bounding_boxes/dragon.obj'... ");
    fflush(stdout);
    construct_group_from_obj_file("scenes/bounding_boxes/dragon.obj", color_space_fn, shape_0_child_1_child_0);
    printf("Done!\n");
    fflush(stdout);

    shape_set_material_recursive(shape_0_child_1_child_0, material_0_child_1_child_0);
    shape_set_transform(shape_0_child_1_child_0, transform_0_child_1_child_0);


    
        Pattern pattern_0_child_1_child_1_Ka = NULL;
    Pattern pattern_0_child_1_child_1_Kd = NULL;
    Pattern pattern_0_child_1_child_1_Ks = NULL;
    Pattern pattern_0_child_1_child_1_Ns = NULL;
    Pattern pattern_0_child_1_child_1_bump = NULL;
    Pattern pattern_0_child_1_child_1_disp = NULL;
    Pattern pattern_0_child_1_child_1_refl = NULL;
    Pattern pattern_0_child_1_child_1_d = NULL;
    Color material_0_child_1_child_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_0_child_1_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_child_1_child_1_refractive = color(0.9000000000, 0.9000000000, 0.9000000000);

    Material material_0_child_1_child_1 = material_alloc();
    color_space_fn(material_0_child_1_child_1_color_raw, material_0_child_1_child_1->Ka);
    color_space_fn(material_0_child_1_child_1_color_raw, material_0_child_1_child_1->Kd);
    color_space_fn(material_0_child_1_child_1_color_raw, material_0_child_1_child_1->Ks);
    color_scale(material_0_child_1_child_1->Ka, 0.0000000000);
    color_scale(material_0_child_1_child_1->Kd, 0.4000000000);
    color_scale(material_0_child_1_child_1->Ks, 0.0000000000);
    rgb_to_rgb(material_0_child_1_child_1_reflective, material_0_child_1_child_1->refl);
    rgb_to_rgb(material_0_child_1_child_1_refractive, material_0_child_1_child_1->Tf);
    material_0_child_1_child_1->reflective = material_0_child_1_child_1_reflective[0] > 0.0
                             || material_0_child_1_child_1_reflective[1] > 0.0
                             || material_0_child_1_child_1_reflective[2] > 0.0;

    material_0_child_1_child_1->Tr = 0.9000000000;
    material_0_child_1_child_1->Ns = 200.0000000000;
    material_0_child_1_child_1->Ni = 1.0000000000;
    material_0_child_1_child_1->casts_shadow = false;
    material_set_pattern(material_0_child_1_child_1, map_Ka, pattern_0_child_1_child_1_Ka);
    material_set_pattern(material_0_child_1_child_1, map_Kd, pattern_0_child_1_child_1_Kd);
    material_set_pattern(material_0_child_1_child_1, map_Ks, pattern_0_child_1_child_1_Ks);
    material_set_pattern(material_0_child_1_child_1, map_Ns, pattern_0_child_1_child_1_Ns);
    material_set_pattern(material_0_child_1_child_1, map_d, pattern_0_child_1_child_1_d);
    material_set_pattern(material_0_child_1_child_1, map_bump, pattern_0_child_1_child_1_bump);
    material_set_pattern(material_0_child_1_child_1, map_disp, pattern_0_child_1_child_1_disp);
    material_set_pattern(material_0_child_1_child_1, map_refl, pattern_0_child_1_child_1_refl);

    Matrix transform_0_child_1_child_1, transform_0_child_1_child_1_tmp;
    matrix_identity(transform_0_child_1_child_1);
    matrix_translate(1.0000000000, 1.0000000000, 1.0000000000, transform_0_child_1_child_1_tmp);
    transform_chain(transform_0_child_1_child_1_tmp, transform_0_child_1_child_1);
    matrix_scale(3.7333500000, 2.5845000000, 1.6283000000, transform_0_child_1_child_1_tmp);
    transform_chain(transform_0_child_1_child_1_tmp, transform_0_child_1_child_1);
    matrix_translate(-3.9863000000, -0.1217000000, -1.1820000000, transform_0_child_1_child_1_tmp);
    transform_chain(transform_0_child_1_child_1_tmp, transform_0_child_1_child_1);
    matrix_translate(0.0000000000, 0.1216900000, 0.0000000000, transform_0_child_1_child_1_tmp);
    transform_chain(transform_0_child_1_child_1_tmp, transform_0_child_1_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_0_child_1_child_1_tmp);
    transform_chain(transform_0_child_1_child_1_tmp, transform_0_child_1_child_1);

    Shape shape_0_child_1_child_1 = shape_0_child_1_children + 1;
    cube(shape_0_child_1_child_1);
    shape_set_material(shape_0_child_1_child_1, material_0_child_1_child_1);
    shape_set_transform(shape_0_child_1_child_1, transform_0_child_1_child_1);

    /* end children for 0_child_1 */

    Matrix transform_0_child_1;
    matrix_identity(transform_0_child_1);
    Shape shape_0_child_1 = shape_0_children + 1;
    group(shape_0_child_1, shape_0_child_1_children, 2);
    //shape_free(shape_0_child_1_children);
    shape_set_transform(shape_0_child_1, transform_0_child_1);

    /* end children for 0 */

    Matrix transform_0;
    matrix_translate(0.0000000000, 2.0000000000, 0.0000000000, transform_0);
    Shape shape_0 = all_shapes + 0;
    group(shape_0, shape_0_children, 2);
    //shape_free(shape_0_children);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* shape 1 */
    
    /* children for 1 */
    Shape shape_1_children = array_of_shapes(2);

    
        Pattern pattern_1_child_0_Ka = NULL;
    Pattern pattern_1_child_0_Kd = NULL;
    Pattern pattern_1_child_0_Ks = NULL;
    Pattern pattern_1_child_0_Ns = NULL;
    Pattern pattern_1_child_0_bump = NULL;
    Pattern pattern_1_child_0_disp = NULL;
    Pattern pattern_1_child_0_refl = NULL;
    Pattern pattern_1_child_0_d = NULL;
    Color material_1_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_1_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1_child_0 = material_alloc();
    color_space_fn(material_1_child_0_color_raw, material_1_child_0->Ka);
    color_space_fn(material_1_child_0_color_raw, material_1_child_0->Kd);
    color_space_fn(material_1_child_0_color_raw, material_1_child_0->Ks);
    color_scale(material_1_child_0->Ka, 0.0000000000);
    color_scale(material_1_child_0->Kd, 0.8000000000);
    color_scale(material_1_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_1_child_0_reflective, material_1_child_0->refl);
    rgb_to_rgb(material_1_child_0_refractive, material_1_child_0->Tf);
    material_1_child_0->reflective = material_1_child_0_reflective[0] > 0.0
                             || material_1_child_0_reflective[1] > 0.0
                             || material_1_child_0_reflective[2] > 0.0;

    material_1_child_0->Tr = 0.0000000000;
    material_1_child_0->Ns = 200.0000000000;
    material_1_child_0->Ni = 1.0000000000;
    material_1_child_0->casts_shadow = true;
    material_set_pattern(material_1_child_0, map_Ka, pattern_1_child_0_Ka);
    material_set_pattern(material_1_child_0, map_Kd, pattern_1_child_0_Kd);
    material_set_pattern(material_1_child_0, map_Ks, pattern_1_child_0_Ks);
    material_set_pattern(material_1_child_0, map_Ns, pattern_1_child_0_Ns);
    material_set_pattern(material_1_child_0, map_d, pattern_1_child_0_d);
    material_set_pattern(material_1_child_0, map_bump, pattern_1_child_0_bump);
    material_set_pattern(material_1_child_0, map_disp, pattern_1_child_0_disp);
    material_set_pattern(material_1_child_0, map_refl, pattern_1_child_0_refl);

    Matrix transform_1_child_0;
    matrix_identity(transform_1_child_0);
    Shape shape_1_child_0 = shape_1_children + 0;
    cylinder(shape_1_child_0);
    shape_set_material(shape_1_child_0, material_1_child_0);
    shape_set_transform(shape_1_child_0, transform_1_child_0);
    shape_1_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_1_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_1_child_0->fields.cylinder.closed = true;


    
    /* children for 1_child_1 */
    Shape shape_1_child_1_children = array_of_shapes(2);

        Pattern pattern_1_child_1_child_0_Ka = NULL;
    Pattern pattern_1_child_1_child_0_Kd = NULL;
    Pattern pattern_1_child_1_child_0_Ks = NULL;
    Pattern pattern_1_child_1_child_0_Ns = NULL;
    Pattern pattern_1_child_1_child_0_bump = NULL;
    Pattern pattern_1_child_1_child_0_disp = NULL;
    Pattern pattern_1_child_1_child_0_refl = NULL;
    Pattern pattern_1_child_1_child_0_d = NULL;
    Color material_1_child_1_child_0_color_raw = color(1.0000000000, 0.5000000000, 0.1000000000);
    Color material_1_child_1_child_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_child_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1_child_1_child_0 = material_alloc();
    color_space_fn(material_1_child_1_child_0_color_raw, material_1_child_1_child_0->Ka);
    color_space_fn(material_1_child_1_child_0_color_raw, material_1_child_1_child_0->Kd);
    color_space_fn(material_1_child_1_child_0_color_raw, material_1_child_1_child_0->Ks);
    color_scale(material_1_child_1_child_0->Ka, 0.1000000000);
    color_scale(material_1_child_1_child_0->Kd, 0.6000000000);
    color_scale(material_1_child_1_child_0->Ks, 0.8000000000);
    rgb_to_rgb(material_1_child_1_child_0_reflective, material_1_child_1_child_0->refl);
    rgb_to_rgb(material_1_child_1_child_0_refractive, material_1_child_1_child_0->Tf);
    material_1_child_1_child_0->reflective = material_1_child_1_child_0_reflective[0] > 0.0
                             || material_1_child_1_child_0_reflective[1] > 0.0
                             || material_1_child_1_child_0_reflective[2] > 0.0;

    material_1_child_1_child_0->Tr = 0.0000000000;
    material_1_child_1_child_0->Ns = 15.0000000000;
    material_1_child_1_child_0->Ni = 1.0000000000;
    material_1_child_1_child_0->casts_shadow = true;
    material_set_pattern(material_1_child_1_child_0, map_Ka, pattern_1_child_1_child_0_Ka);
    material_set_pattern(material_1_child_1_child_0, map_Kd, pattern_1_child_1_child_0_Kd);
    material_set_pattern(material_1_child_1_child_0, map_Ks, pattern_1_child_1_child_0_Ks);
    material_set_pattern(material_1_child_1_child_0, map_Ns, pattern_1_child_1_child_0_Ns);
    material_set_pattern(material_1_child_1_child_0, map_d, pattern_1_child_1_child_0_d);
    material_set_pattern(material_1_child_1_child_0, map_bump, pattern_1_child_1_child_0_bump);
    material_set_pattern(material_1_child_1_child_0, map_disp, pattern_1_child_1_child_0_disp);
    material_set_pattern(material_1_child_1_child_0, map_refl, pattern_1_child_1_child_0_refl);

    Matrix transform_1_child_1_child_0, transform_1_child_1_child_0_tmp;
    matrix_identity(transform_1_child_1_child_0);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_1_child_1_child_0_tmp);
    transform_chain(transform_1_child_1_child_0_tmp, transform_1_child_1_child_0);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_1_child_1_child_0_tmp);
    transform_chain(transform_1_child_1_child_0_tmp, transform_1_child_1_child_0);

    Shape shape_1_child_1_child_0 = shape_1_child_1_children + 0;
    shape_copy(shape_0_child_1_child_0, NULL, shape_1_child_1_child_0);
    shape_set_material_recursive(shape_1_child_1_child_0, material_1_child_1_child_0);
    shape_set_transform(shape_1_child_1_child_0, transform_1_child_1_child_0);


    
        Pattern pattern_1_child_1_child_1_Ka = NULL;
    Pattern pattern_1_child_1_child_1_Kd = NULL;
    Pattern pattern_1_child_1_child_1_Ks = NULL;
    Pattern pattern_1_child_1_child_1_Ns = NULL;
    Pattern pattern_1_child_1_child_1_bump = NULL;
    Pattern pattern_1_child_1_child_1_disp = NULL;
    Pattern pattern_1_child_1_child_1_refl = NULL;
    Pattern pattern_1_child_1_child_1_d = NULL;
    Color material_1_child_1_child_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_1_child_1_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_child_1_child_1_refractive = color(0.8000000000, 0.8000000000, 0.8000000000);

    Material material_1_child_1_child_1 = material_alloc();
    color_space_fn(material_1_child_1_child_1_color_raw, material_1_child_1_child_1->Ka);
    color_space_fn(material_1_child_1_child_1_color_raw, material_1_child_1_child_1->Kd);
    color_space_fn(material_1_child_1_child_1_color_raw, material_1_child_1_child_1->Ks);
    color_scale(material_1_child_1_child_1->Ka, 0.0000000000);
    color_scale(material_1_child_1_child_1->Kd, 0.2000000000);
    color_scale(material_1_child_1_child_1->Ks, 0.0000000000);
    rgb_to_rgb(material_1_child_1_child_1_reflective, material_1_child_1_child_1->refl);
    rgb_to_rgb(material_1_child_1_child_1_refractive, material_1_child_1_child_1->Tf);
    material_1_child_1_child_1->reflective = material_1_child_1_child_1_reflective[0] > 0.0
                             || material_1_child_1_child_1_reflective[1] > 0.0
                             || material_1_child_1_child_1_reflective[2] > 0.0;

    material_1_child_1_child_1->Tr = 0.8000000000;
    material_1_child_1_child_1->Ns = 200.0000000000;
    material_1_child_1_child_1->Ni = 1.0000000000;
    material_1_child_1_child_1->casts_shadow = false;
    material_set_pattern(material_1_child_1_child_1, map_Ka, pattern_1_child_1_child_1_Ka);
    material_set_pattern(material_1_child_1_child_1, map_Kd, pattern_1_child_1_child_1_Kd);
    material_set_pattern(material_1_child_1_child_1, map_Ks, pattern_1_child_1_child_1_Ks);
    material_set_pattern(material_1_child_1_child_1, map_Ns, pattern_1_child_1_child_1_Ns);
    material_set_pattern(material_1_child_1_child_1, map_d, pattern_1_child_1_child_1_d);
    material_set_pattern(material_1_child_1_child_1, map_bump, pattern_1_child_1_child_1_bump);
    material_set_pattern(material_1_child_1_child_1, map_disp, pattern_1_child_1_child_1_disp);
    material_set_pattern(material_1_child_1_child_1, map_refl, pattern_1_child_1_child_1_refl);

    Matrix transform_1_child_1_child_1, transform_1_child_1_child_1_tmp;
    matrix_identity(transform_1_child_1_child_1);
    matrix_translate(1.0000000000, 1.0000000000, 1.0000000000, transform_1_child_1_child_1_tmp);
    transform_chain(transform_1_child_1_child_1_tmp, transform_1_child_1_child_1);
    matrix_scale(3.7333500000, 2.5845000000, 1.6283000000, transform_1_child_1_child_1_tmp);
    transform_chain(transform_1_child_1_child_1_tmp, transform_1_child_1_child_1);
    matrix_translate(-3.9863000000, -0.1217000000, -1.1820000000, transform_1_child_1_child_1_tmp);
    transform_chain(transform_1_child_1_child_1_tmp, transform_1_child_1_child_1);
    matrix_translate(0.0000000000, 0.1216900000, 0.0000000000, transform_1_child_1_child_1_tmp);
    transform_chain(transform_1_child_1_child_1_tmp, transform_1_child_1_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_1_child_1_child_1_tmp);
    transform_chain(transform_1_child_1_child_1_tmp, transform_1_child_1_child_1);

    Shape shape_1_child_1_child_1 = shape_1_child_1_children + 1;
    cube(shape_1_child_1_child_1);
    shape_set_material(shape_1_child_1_child_1, material_1_child_1_child_1);
    shape_set_transform(shape_1_child_1_child_1, transform_1_child_1_child_1);

    /* end children for 1_child_1 */

    Matrix transform_1_child_1, transform_1_child_1_tmp;
    matrix_identity(transform_1_child_1);
    matrix_rotate_y(4.0000000000, transform_1_child_1_tmp);
    transform_chain(transform_1_child_1_tmp, transform_1_child_1);
    matrix_scale(0.7500000000, 0.7500000000, 0.7500000000, transform_1_child_1_tmp);
    transform_chain(transform_1_child_1_tmp, transform_1_child_1);

    Shape shape_1_child_1 = shape_1_children + 1;
    group(shape_1_child_1, shape_1_child_1_children, 2);
    //shape_free(shape_1_child_1_children);
    shape_set_transform(shape_1_child_1, transform_1_child_1);

    /* end children for 1 */

    Matrix transform_1;
    matrix_translate(2.0000000000, 1.0000000000, -1.0000000000, transform_1);
    Shape shape_1 = all_shapes + 1;
    group(shape_1, shape_1_children, 2);
    //shape_free(shape_1_children);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* shape 2 */
    
    /* children for 2 */
    Shape shape_2_children = array_of_shapes(2);

    
        Pattern pattern_2_child_0_Ka = NULL;
    Pattern pattern_2_child_0_Kd = NULL;
    Pattern pattern_2_child_0_Ks = NULL;
    Pattern pattern_2_child_0_Ns = NULL;
    Pattern pattern_2_child_0_bump = NULL;
    Pattern pattern_2_child_0_disp = NULL;
    Pattern pattern_2_child_0_refl = NULL;
    Pattern pattern_2_child_0_d = NULL;
    Color material_2_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_2_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_2_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2_child_0 = material_alloc();
    color_space_fn(material_2_child_0_color_raw, material_2_child_0->Ka);
    color_space_fn(material_2_child_0_color_raw, material_2_child_0->Kd);
    color_space_fn(material_2_child_0_color_raw, material_2_child_0->Ks);
    color_scale(material_2_child_0->Ka, 0.0000000000);
    color_scale(material_2_child_0->Kd, 0.8000000000);
    color_scale(material_2_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_2_child_0_reflective, material_2_child_0->refl);
    rgb_to_rgb(material_2_child_0_refractive, material_2_child_0->Tf);
    material_2_child_0->reflective = material_2_child_0_reflective[0] > 0.0
                             || material_2_child_0_reflective[1] > 0.0
                             || material_2_child_0_reflective[2] > 0.0;

    material_2_child_0->Tr = 0.0000000000;
    material_2_child_0->Ns = 200.0000000000;
    material_2_child_0->Ni = 1.0000000000;
    material_2_child_0->casts_shadow = true;
    material_set_pattern(material_2_child_0, map_Ka, pattern_2_child_0_Ka);
    material_set_pattern(material_2_child_0, map_Kd, pattern_2_child_0_Kd);
    material_set_pattern(material_2_child_0, map_Ks, pattern_2_child_0_Ks);
    material_set_pattern(material_2_child_0, map_Ns, pattern_2_child_0_Ns);
    material_set_pattern(material_2_child_0, map_d, pattern_2_child_0_d);
    material_set_pattern(material_2_child_0, map_bump, pattern_2_child_0_bump);
    material_set_pattern(material_2_child_0, map_disp, pattern_2_child_0_disp);
    material_set_pattern(material_2_child_0, map_refl, pattern_2_child_0_refl);

    Matrix transform_2_child_0;
    matrix_identity(transform_2_child_0);
    Shape shape_2_child_0 = shape_2_children + 0;
    cylinder(shape_2_child_0);
    shape_set_material(shape_2_child_0, material_2_child_0);
    shape_set_transform(shape_2_child_0, transform_2_child_0);
    shape_2_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_2_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_2_child_0->fields.cylinder.closed = true;


    
    /* children for 2_child_1 */
    Shape shape_2_child_1_children = array_of_shapes(2);

        Pattern pattern_2_child_1_child_0_Ka = NULL;
    Pattern pattern_2_child_1_child_0_Kd = NULL;
    Pattern pattern_2_child_1_child_0_Ks = NULL;
    Pattern pattern_2_child_1_child_0_Ns = NULL;
    Pattern pattern_2_child_1_child_0_bump = NULL;
    Pattern pattern_2_child_1_child_0_disp = NULL;
    Pattern pattern_2_child_1_child_0_refl = NULL;
    Pattern pattern_2_child_1_child_0_d = NULL;
    Color material_2_child_1_child_0_color_raw = color(0.9000000000, 0.5000000000, 0.1000000000);
    Color material_2_child_1_child_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_2_child_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_2_child_1_child_0 = material_alloc();
    color_space_fn(material_2_child_1_child_0_color_raw, material_2_child_1_child_0->Ka);
    color_space_fn(material_2_child_1_child_0_color_raw, material_2_child_1_child_0->Kd);
    color_space_fn(material_2_child_1_child_0_color_raw, material_2_child_1_child_0->Ks);
    color_scale(material_2_child_1_child_0->Ka, 0.1000000000);
    color_scale(material_2_child_1_child_0->Kd, 0.6000000000);
    color_scale(material_2_child_1_child_0->Ks, 0.8000000000);
    rgb_to_rgb(material_2_child_1_child_0_reflective, material_2_child_1_child_0->refl);
    rgb_to_rgb(material_2_child_1_child_0_refractive, material_2_child_1_child_0->Tf);
    material_2_child_1_child_0->reflective = material_2_child_1_child_0_reflective[0] > 0.0
                             || material_2_child_1_child_0_reflective[1] > 0.0
                             || material_2_child_1_child_0_reflective[2] > 0.0;

    material_2_child_1_child_0->Tr = 0.0000000000;
    material_2_child_1_child_0->Ns = 15.0000000000;
    material_2_child_1_child_0->Ni = 1.0000000000;
    material_2_child_1_child_0->casts_shadow = true;
    material_set_pattern(material_2_child_1_child_0, map_Ka, pattern_2_child_1_child_0_Ka);
    material_set_pattern(material_2_child_1_child_0, map_Kd, pattern_2_child_1_child_0_Kd);
    material_set_pattern(material_2_child_1_child_0, map_Ks, pattern_2_child_1_child_0_Ks);
    material_set_pattern(material_2_child_1_child_0, map_Ns, pattern_2_child_1_child_0_Ns);
    material_set_pattern(material_2_child_1_child_0, map_d, pattern_2_child_1_child_0_d);
    material_set_pattern(material_2_child_1_child_0, map_bump, pattern_2_child_1_child_0_bump);
    material_set_pattern(material_2_child_1_child_0, map_disp, pattern_2_child_1_child_0_disp);
    material_set_pattern(material_2_child_1_child_0, map_refl, pattern_2_child_1_child_0_refl);

    Matrix transform_2_child_1_child_0, transform_2_child_1_child_0_tmp;
    matrix_identity(transform_2_child_1_child_0);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_2_child_1_child_0_tmp);
    transform_chain(transform_2_child_1_child_0_tmp, transform_2_child_1_child_0);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_2_child_1_child_0_tmp);
    transform_chain(transform_2_child_1_child_0_tmp, transform_2_child_1_child_0);

    Shape shape_2_child_1_child_0 = shape_2_child_1_children + 0;
    shape_copy(shape_1_child_1_child_0, NULL, shape_2_child_1_child_0);
    shape_set_material_recursive(shape_2_child_1_child_0, material_2_child_1_child_0);
    shape_set_transform(shape_2_child_1_child_0, transform_2_child_1_child_0);


    
        Pattern pattern_2_child_1_child_1_Ka = NULL;
    Pattern pattern_2_child_1_child_1_Kd = NULL;
    Pattern pattern_2_child_1_child_1_Ks = NULL;
    Pattern pattern_2_child_1_child_1_Ns = NULL;
    Pattern pattern_2_child_1_child_1_bump = NULL;
    Pattern pattern_2_child_1_child_1_disp = NULL;
    Pattern pattern_2_child_1_child_1_refl = NULL;
    Pattern pattern_2_child_1_child_1_d = NULL;
    Color material_2_child_1_child_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_2_child_1_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_2_child_1_child_1_refractive = color(0.8000000000, 0.8000000000, 0.8000000000);

    Material material_2_child_1_child_1 = material_alloc();
    color_space_fn(material_2_child_1_child_1_color_raw, material_2_child_1_child_1->Ka);
    color_space_fn(material_2_child_1_child_1_color_raw, material_2_child_1_child_1->Kd);
    color_space_fn(material_2_child_1_child_1_color_raw, material_2_child_1_child_1->Ks);
    color_scale(material_2_child_1_child_1->Ka, 0.0000000000);
    color_scale(material_2_child_1_child_1->Kd, 0.2000000000);
    color_scale(material_2_child_1_child_1->Ks, 0.0000000000);
    rgb_to_rgb(material_2_child_1_child_1_reflective, material_2_child_1_child_1->refl);
    rgb_to_rgb(material_2_child_1_child_1_refractive, material_2_child_1_child_1->Tf);
    material_2_child_1_child_1->reflective = material_2_child_1_child_1_reflective[0] > 0.0
                             || material_2_child_1_child_1_reflective[1] > 0.0
                             || material_2_child_1_child_1_reflective[2] > 0.0;

    material_2_child_1_child_1->Tr = 0.8000000000;
    material_2_child_1_child_1->Ns = 200.0000000000;
    material_2_child_1_child_1->Ni = 1.0000000000;
    material_2_child_1_child_1->casts_shadow = false;
    material_set_pattern(material_2_child_1_child_1, map_Ka, pattern_2_child_1_child_1_Ka);
    material_set_pattern(material_2_child_1_child_1, map_Kd, pattern_2_child_1_child_1_Kd);
    material_set_pattern(material_2_child_1_child_1, map_Ks, pattern_2_child_1_child_1_Ks);
    material_set_pattern(material_2_child_1_child_1, map_Ns, pattern_2_child_1_child_1_Ns);
    material_set_pattern(material_2_child_1_child_1, map_d, pattern_2_child_1_child_1_d);
    material_set_pattern(material_2_child_1_child_1, map_bump, pattern_2_child_1_child_1_bump);
    material_set_pattern(material_2_child_1_child_1, map_disp, pattern_2_child_1_child_1_disp);
    material_set_pattern(material_2_child_1_child_1, map_refl, pattern_2_child_1_child_1_refl);

    Matrix transform_2_child_1_child_1, transform_2_child_1_child_1_tmp;
    matrix_identity(transform_2_child_1_child_1);
    matrix_translate(1.0000000000, 1.0000000000, 1.0000000000, transform_2_child_1_child_1_tmp);
    transform_chain(transform_2_child_1_child_1_tmp, transform_2_child_1_child_1);
    matrix_scale(3.7333500000, 2.5845000000, 1.6283000000, transform_2_child_1_child_1_tmp);
    transform_chain(transform_2_child_1_child_1_tmp, transform_2_child_1_child_1);
    matrix_translate(-3.9863000000, -0.1217000000, -1.1820000000, transform_2_child_1_child_1_tmp);
    transform_chain(transform_2_child_1_child_1_tmp, transform_2_child_1_child_1);
    matrix_translate(0.0000000000, 0.1216900000, 0.0000000000, transform_2_child_1_child_1_tmp);
    transform_chain(transform_2_child_1_child_1_tmp, transform_2_child_1_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_2_child_1_child_1_tmp);
    transform_chain(transform_2_child_1_child_1_tmp, transform_2_child_1_child_1);

    Shape shape_2_child_1_child_1 = shape_2_child_1_children + 1;
    cube(shape_2_child_1_child_1);
    shape_set_material(shape_2_child_1_child_1, material_2_child_1_child_1);
    shape_set_transform(shape_2_child_1_child_1, transform_2_child_1_child_1);

    /* end children for 2_child_1 */

    Matrix transform_2_child_1, transform_2_child_1_tmp;
    matrix_identity(transform_2_child_1);
    matrix_rotate_y(-0.4000000000, transform_2_child_1_tmp);
    transform_chain(transform_2_child_1_tmp, transform_2_child_1);
    matrix_scale(0.7500000000, 0.7500000000, 0.7500000000, transform_2_child_1_tmp);
    transform_chain(transform_2_child_1_tmp, transform_2_child_1);

    Shape shape_2_child_1 = shape_2_children + 1;
    group(shape_2_child_1, shape_2_child_1_children, 2);
    //shape_free(shape_2_child_1_children);
    shape_set_transform(shape_2_child_1, transform_2_child_1);

    /* end children for 2 */

    Matrix transform_2;
    matrix_translate(-2.0000000000, 0.7500000000, -1.0000000000, transform_2);
    Shape shape_2 = all_shapes + 2;
    group(shape_2, shape_2_children, 2);
    //shape_free(shape_2_children);
    shape_set_transform(shape_2, transform_2);

    /* end shape 2 */
    /* shape 3 */
    
    /* children for 3 */
    Shape shape_3_children = array_of_shapes(2);

    
        Pattern pattern_3_child_0_Ka = NULL;
    Pattern pattern_3_child_0_Kd = NULL;
    Pattern pattern_3_child_0_Ks = NULL;
    Pattern pattern_3_child_0_Ns = NULL;
    Pattern pattern_3_child_0_bump = NULL;
    Pattern pattern_3_child_0_disp = NULL;
    Pattern pattern_3_child_0_refl = NULL;
    Pattern pattern_3_child_0_d = NULL;
    Color material_3_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_3_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_3_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3_child_0 = material_alloc();
    color_space_fn(material_3_child_0_color_raw, material_3_child_0->Ka);
    color_space_fn(material_3_child_0_color_raw, material_3_child_0->Kd);
    color_space_fn(material_3_child_0_color_raw, material_3_child_0->Ks);
    color_scale(material_3_child_0->Ka, 0.0000000000);
    color_scale(material_3_child_0->Kd, 0.8000000000);
    color_scale(material_3_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_3_child_0_reflective, material_3_child_0->refl);
    rgb_to_rgb(material_3_child_0_refractive, material_3_child_0->Tf);
    material_3_child_0->reflective = material_3_child_0_reflective[0] > 0.0
                             || material_3_child_0_reflective[1] > 0.0
                             || material_3_child_0_reflective[2] > 0.0;

    material_3_child_0->Tr = 0.0000000000;
    material_3_child_0->Ns = 200.0000000000;
    material_3_child_0->Ni = 1.0000000000;
    material_3_child_0->casts_shadow = true;
    material_set_pattern(material_3_child_0, map_Ka, pattern_3_child_0_Ka);
    material_set_pattern(material_3_child_0, map_Kd, pattern_3_child_0_Kd);
    material_set_pattern(material_3_child_0, map_Ks, pattern_3_child_0_Ks);
    material_set_pattern(material_3_child_0, map_Ns, pattern_3_child_0_Ns);
    material_set_pattern(material_3_child_0, map_d, pattern_3_child_0_d);
    material_set_pattern(material_3_child_0, map_bump, pattern_3_child_0_bump);
    material_set_pattern(material_3_child_0, map_disp, pattern_3_child_0_disp);
    material_set_pattern(material_3_child_0, map_refl, pattern_3_child_0_refl);

    Matrix transform_3_child_0;
    matrix_identity(transform_3_child_0);
    Shape shape_3_child_0 = shape_3_children + 0;
    cylinder(shape_3_child_0);
    shape_set_material(shape_3_child_0, material_3_child_0);
    shape_set_transform(shape_3_child_0, transform_3_child_0);
    shape_3_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_3_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_3_child_0->fields.cylinder.closed = true;


    
    /* children for 3_child_1 */
    Shape shape_3_child_1_children = array_of_shapes(2);

        Pattern pattern_3_child_1_child_0_Ka = NULL;
    Pattern pattern_3_child_1_child_0_Kd = NULL;
    Pattern pattern_3_child_1_child_0_Ks = NULL;
    Pattern pattern_3_child_1_child_0_Ns = NULL;
    Pattern pattern_3_child_1_child_0_bump = NULL;
    Pattern pattern_3_child_1_child_0_disp = NULL;
    Pattern pattern_3_child_1_child_0_refl = NULL;
    Pattern pattern_3_child_1_child_0_d = NULL;
    Color material_3_child_1_child_0_color_raw = color(1.0000000000, 0.9000000000, 0.1000000000);
    Color material_3_child_1_child_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_3_child_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_3_child_1_child_0 = material_alloc();
    color_space_fn(material_3_child_1_child_0_color_raw, material_3_child_1_child_0->Ka);
    color_space_fn(material_3_child_1_child_0_color_raw, material_3_child_1_child_0->Kd);
    color_space_fn(material_3_child_1_child_0_color_raw, material_3_child_1_child_0->Ks);
    color_scale(material_3_child_1_child_0->Ka, 0.1000000000);
    color_scale(material_3_child_1_child_0->Kd, 0.6000000000);
    color_scale(material_3_child_1_child_0->Ks, 0.8000000000);
    rgb_to_rgb(material_3_child_1_child_0_reflective, material_3_child_1_child_0->refl);
    rgb_to_rgb(material_3_child_1_child_0_refractive, material_3_child_1_child_0->Tf);
    material_3_child_1_child_0->reflective = material_3_child_1_child_0_reflective[0] > 0.0
                             || material_3_child_1_child_0_reflective[1] > 0.0
                             || material_3_child_1_child_0_reflective[2] > 0.0;

    material_3_child_1_child_0->Tr = 0.0000000000;
    material_3_child_1_child_0->Ns = 15.0000000000;
    material_3_child_1_child_0->Ni = 1.0000000000;
    material_3_child_1_child_0->casts_shadow = true;
    material_set_pattern(material_3_child_1_child_0, map_Ka, pattern_3_child_1_child_0_Ka);
    material_set_pattern(material_3_child_1_child_0, map_Kd, pattern_3_child_1_child_0_Kd);
    material_set_pattern(material_3_child_1_child_0, map_Ks, pattern_3_child_1_child_0_Ks);
    material_set_pattern(material_3_child_1_child_0, map_Ns, pattern_3_child_1_child_0_Ns);
    material_set_pattern(material_3_child_1_child_0, map_d, pattern_3_child_1_child_0_d);
    material_set_pattern(material_3_child_1_child_0, map_bump, pattern_3_child_1_child_0_bump);
    material_set_pattern(material_3_child_1_child_0, map_disp, pattern_3_child_1_child_0_disp);
    material_set_pattern(material_3_child_1_child_0, map_refl, pattern_3_child_1_child_0_refl);

    Matrix transform_3_child_1_child_0, transform_3_child_1_child_0_tmp;
    matrix_identity(transform_3_child_1_child_0);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_3_child_1_child_0_tmp);
    transform_chain(transform_3_child_1_child_0_tmp, transform_3_child_1_child_0);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_3_child_1_child_0_tmp);
    transform_chain(transform_3_child_1_child_0_tmp, transform_3_child_1_child_0);

    Shape shape_3_child_1_child_0 = shape_3_child_1_children + 0;
    shape_copy(shape_2_child_1_child_0, NULL, shape_3_child_1_child_0);
    shape_set_material_recursive(shape_3_child_1_child_0, material_3_child_1_child_0);
    shape_set_transform(shape_3_child_1_child_0, transform_3_child_1_child_0);


    
        Pattern pattern_3_child_1_child_1_Ka = NULL;
    Pattern pattern_3_child_1_child_1_Kd = NULL;
    Pattern pattern_3_child_1_child_1_Ks = NULL;
    Pattern pattern_3_child_1_child_1_Ns = NULL;
    Pattern pattern_3_child_1_child_1_bump = NULL;
    Pattern pattern_3_child_1_child_1_disp = NULL;
    Pattern pattern_3_child_1_child_1_refl = NULL;
    Pattern pattern_3_child_1_child_1_d = NULL;
    Color material_3_child_1_child_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_3_child_1_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_3_child_1_child_1_refractive = color(0.9000000000, 0.9000000000, 0.9000000000);

    Material material_3_child_1_child_1 = material_alloc();
    color_space_fn(material_3_child_1_child_1_color_raw, material_3_child_1_child_1->Ka);
    color_space_fn(material_3_child_1_child_1_color_raw, material_3_child_1_child_1->Kd);
    color_space_fn(material_3_child_1_child_1_color_raw, material_3_child_1_child_1->Ks);
    color_scale(material_3_child_1_child_1->Ka, 0.0000000000);
    color_scale(material_3_child_1_child_1->Kd, 0.1000000000);
    color_scale(material_3_child_1_child_1->Ks, 0.0000000000);
    rgb_to_rgb(material_3_child_1_child_1_reflective, material_3_child_1_child_1->refl);
    rgb_to_rgb(material_3_child_1_child_1_refractive, material_3_child_1_child_1->Tf);
    material_3_child_1_child_1->reflective = material_3_child_1_child_1_reflective[0] > 0.0
                             || material_3_child_1_child_1_reflective[1] > 0.0
                             || material_3_child_1_child_1_reflective[2] > 0.0;

    material_3_child_1_child_1->Tr = 0.9000000000;
    material_3_child_1_child_1->Ns = 200.0000000000;
    material_3_child_1_child_1->Ni = 1.0000000000;
    material_3_child_1_child_1->casts_shadow = false;
    material_set_pattern(material_3_child_1_child_1, map_Ka, pattern_3_child_1_child_1_Ka);
    material_set_pattern(material_3_child_1_child_1, map_Kd, pattern_3_child_1_child_1_Kd);
    material_set_pattern(material_3_child_1_child_1, map_Ks, pattern_3_child_1_child_1_Ks);
    material_set_pattern(material_3_child_1_child_1, map_Ns, pattern_3_child_1_child_1_Ns);
    material_set_pattern(material_3_child_1_child_1, map_d, pattern_3_child_1_child_1_d);
    material_set_pattern(material_3_child_1_child_1, map_bump, pattern_3_child_1_child_1_bump);
    material_set_pattern(material_3_child_1_child_1, map_disp, pattern_3_child_1_child_1_disp);
    material_set_pattern(material_3_child_1_child_1, map_refl, pattern_3_child_1_child_1_refl);

    Matrix transform_3_child_1_child_1, transform_3_child_1_child_1_tmp;
    matrix_identity(transform_3_child_1_child_1);
    matrix_translate(1.0000000000, 1.0000000000, 1.0000000000, transform_3_child_1_child_1_tmp);
    transform_chain(transform_3_child_1_child_1_tmp, transform_3_child_1_child_1);
    matrix_scale(3.7333500000, 2.5845000000, 1.6283000000, transform_3_child_1_child_1_tmp);
    transform_chain(transform_3_child_1_child_1_tmp, transform_3_child_1_child_1);
    matrix_translate(-3.9863000000, -0.1217000000, -1.1820000000, transform_3_child_1_child_1_tmp);
    transform_chain(transform_3_child_1_child_1_tmp, transform_3_child_1_child_1);
    matrix_translate(0.0000000000, 0.1216900000, 0.0000000000, transform_3_child_1_child_1_tmp);
    transform_chain(transform_3_child_1_child_1_tmp, transform_3_child_1_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_3_child_1_child_1_tmp);
    transform_chain(transform_3_child_1_child_1_tmp, transform_3_child_1_child_1);

    Shape shape_3_child_1_child_1 = shape_3_child_1_children + 1;
    cube(shape_3_child_1_child_1);
    shape_set_material(shape_3_child_1_child_1, material_3_child_1_child_1);
    shape_set_transform(shape_3_child_1_child_1, transform_3_child_1_child_1);

    /* end children for 3_child_1 */

    Matrix transform_3_child_1, transform_3_child_1_tmp;
    matrix_identity(transform_3_child_1);
    matrix_rotate_y(-0.2000000000, transform_3_child_1_tmp);
    transform_chain(transform_3_child_1_tmp, transform_3_child_1);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_3_child_1_tmp);
    transform_chain(transform_3_child_1_tmp, transform_3_child_1);

    Shape shape_3_child_1 = shape_3_children + 1;
    group(shape_3_child_1, shape_3_child_1_children, 2);
    //shape_free(shape_3_child_1_children);
    shape_set_transform(shape_3_child_1, transform_3_child_1);

    /* end children for 3 */

    Matrix transform_3;
    matrix_translate(-4.0000000000, 0.0000000000, -2.0000000000, transform_3);
    Shape shape_3 = all_shapes + 3;
    group(shape_3, shape_3_children, 2);
    //shape_free(shape_3_children);
    shape_set_transform(shape_3, transform_3);

    /* end shape 3 */
    /* shape 4 */
    
    /* children for 4 */
    Shape shape_4_children = array_of_shapes(2);

    
        Pattern pattern_4_child_0_Ka = NULL;
    Pattern pattern_4_child_0_Kd = NULL;
    Pattern pattern_4_child_0_Ks = NULL;
    Pattern pattern_4_child_0_Ns = NULL;
    Pattern pattern_4_child_0_bump = NULL;
    Pattern pattern_4_child_0_disp = NULL;
    Pattern pattern_4_child_0_refl = NULL;
    Pattern pattern_4_child_0_d = NULL;
    Color material_4_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_4_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_4_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_4_child_0 = material_alloc();
    color_space_fn(material_4_child_0_color_raw, material_4_child_0->Ka);
    color_space_fn(material_4_child_0_color_raw, material_4_child_0->Kd);
    color_space_fn(material_4_child_0_color_raw, material_4_child_0->Ks);
    color_scale(material_4_child_0->Ka, 0.0000000000);
    color_scale(material_4_child_0->Kd, 0.8000000000);
    color_scale(material_4_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_4_child_0_reflective, material_4_child_0->refl);
    rgb_to_rgb(material_4_child_0_refractive, material_4_child_0->Tf);
    material_4_child_0->reflective = material_4_child_0_reflective[0] > 0.0
                             || material_4_child_0_reflective[1] > 0.0
                             || material_4_child_0_reflective[2] > 0.0;

    material_4_child_0->Tr = 0.0000000000;
    material_4_child_0->Ns = 200.0000000000;
    material_4_child_0->Ni = 1.0000000000;
    material_4_child_0->casts_shadow = true;
    material_set_pattern(material_4_child_0, map_Ka, pattern_4_child_0_Ka);
    material_set_pattern(material_4_child_0, map_Kd, pattern_4_child_0_Kd);
    material_set_pattern(material_4_child_0, map_Ks, pattern_4_child_0_Ks);
    material_set_pattern(material_4_child_0, map_Ns, pattern_4_child_0_Ns);
    material_set_pattern(material_4_child_0, map_d, pattern_4_child_0_d);
    material_set_pattern(material_4_child_0, map_bump, pattern_4_child_0_bump);
    material_set_pattern(material_4_child_0, map_disp, pattern_4_child_0_disp);
    material_set_pattern(material_4_child_0, map_refl, pattern_4_child_0_refl);

    Matrix transform_4_child_0;
    matrix_identity(transform_4_child_0);
    Shape shape_4_child_0 = shape_4_children + 0;
    cylinder(shape_4_child_0);
    shape_set_material(shape_4_child_0, material_4_child_0);
    shape_set_transform(shape_4_child_0, transform_4_child_0);
    shape_4_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_4_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_4_child_0->fields.cylinder.closed = true;


    
    /* children for 4_child_1 */
    Shape shape_4_child_1_children = array_of_shapes(2);

        Pattern pattern_4_child_1_child_0_Ka = NULL;
    Pattern pattern_4_child_1_child_0_Kd = NULL;
    Pattern pattern_4_child_1_child_0_Ks = NULL;
    Pattern pattern_4_child_1_child_0_Ns = NULL;
    Pattern pattern_4_child_1_child_0_bump = NULL;
    Pattern pattern_4_child_1_child_0_disp = NULL;
    Pattern pattern_4_child_1_child_0_refl = NULL;
    Pattern pattern_4_child_1_child_0_d = NULL;
    Color material_4_child_1_child_0_color_raw = color(0.9000000000, 1.0000000000, 0.1000000000);
    Color material_4_child_1_child_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_4_child_1_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_4_child_1_child_0 = material_alloc();
    color_space_fn(material_4_child_1_child_0_color_raw, material_4_child_1_child_0->Ka);
    color_space_fn(material_4_child_1_child_0_color_raw, material_4_child_1_child_0->Kd);
    color_space_fn(material_4_child_1_child_0_color_raw, material_4_child_1_child_0->Ks);
    color_scale(material_4_child_1_child_0->Ka, 0.1000000000);
    color_scale(material_4_child_1_child_0->Kd, 0.6000000000);
    color_scale(material_4_child_1_child_0->Ks, 0.8000000000);
    rgb_to_rgb(material_4_child_1_child_0_reflective, material_4_child_1_child_0->refl);
    rgb_to_rgb(material_4_child_1_child_0_refractive, material_4_child_1_child_0->Tf);
    material_4_child_1_child_0->reflective = material_4_child_1_child_0_reflective[0] > 0.0
                             || material_4_child_1_child_0_reflective[1] > 0.0
                             || material_4_child_1_child_0_reflective[2] > 0.0;

    material_4_child_1_child_0->Tr = 0.0000000000;
    material_4_child_1_child_0->Ns = 15.0000000000;
    material_4_child_1_child_0->Ni = 1.0000000000;
    material_4_child_1_child_0->casts_shadow = true;
    material_set_pattern(material_4_child_1_child_0, map_Ka, pattern_4_child_1_child_0_Ka);
    material_set_pattern(material_4_child_1_child_0, map_Kd, pattern_4_child_1_child_0_Kd);
    material_set_pattern(material_4_child_1_child_0, map_Ks, pattern_4_child_1_child_0_Ks);
    material_set_pattern(material_4_child_1_child_0, map_Ns, pattern_4_child_1_child_0_Ns);
    material_set_pattern(material_4_child_1_child_0, map_d, pattern_4_child_1_child_0_d);
    material_set_pattern(material_4_child_1_child_0, map_bump, pattern_4_child_1_child_0_bump);
    material_set_pattern(material_4_child_1_child_0, map_disp, pattern_4_child_1_child_0_disp);
    material_set_pattern(material_4_child_1_child_0, map_refl, pattern_4_child_1_child_0_refl);

    Matrix transform_4_child_1_child_0, transform_4_child_1_child_0_tmp;
    matrix_identity(transform_4_child_1_child_0);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_4_child_1_child_0_tmp);
    transform_chain(transform_4_child_1_child_0_tmp, transform_4_child_1_child_0);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_4_child_1_child_0_tmp);
    transform_chain(transform_4_child_1_child_0_tmp, transform_4_child_1_child_0);

    Shape shape_4_child_1_child_0 = shape_4_child_1_children + 0;
    shape_copy(shape_3_child_1_child_0, NULL, shape_4_child_1_child_0);
    shape_set_material_recursive(shape_4_child_1_child_0, material_4_child_1_child_0);
    shape_set_transform(shape_4_child_1_child_0, transform_4_child_1_child_0);


    
        Pattern pattern_4_child_1_child_1_Ka = NULL;
    Pattern pattern_4_child_1_child_1_Kd = NULL;
    Pattern pattern_4_child_1_child_1_Ks = NULL;
    Pattern pattern_4_child_1_child_1_Ns = NULL;
    Pattern pattern_4_child_1_child_1_bump = NULL;
    Pattern pattern_4_child_1_child_1_disp = NULL;
    Pattern pattern_4_child_1_child_1_refl = NULL;
    Pattern pattern_4_child_1_child_1_d = NULL;
    Color material_4_child_1_child_1_color_raw = color(0.8000000000, 0.8000000000, 0.8000000000);
    Color material_4_child_1_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_4_child_1_child_1_refractive = color(0.9000000000, 0.9000000000, 0.9000000000);

    Material material_4_child_1_child_1 = material_alloc();
    color_space_fn(material_4_child_1_child_1_color_raw, material_4_child_1_child_1->Ka);
    color_space_fn(material_4_child_1_child_1_color_raw, material_4_child_1_child_1->Kd);
    color_space_fn(material_4_child_1_child_1_color_raw, material_4_child_1_child_1->Ks);
    color_scale(material_4_child_1_child_1->Ka, 0.0000000000);
    color_scale(material_4_child_1_child_1->Kd, 0.1000000000);
    color_scale(material_4_child_1_child_1->Ks, 0.0000000000);
    rgb_to_rgb(material_4_child_1_child_1_reflective, material_4_child_1_child_1->refl);
    rgb_to_rgb(material_4_child_1_child_1_refractive, material_4_child_1_child_1->Tf);
    material_4_child_1_child_1->reflective = material_4_child_1_child_1_reflective[0] > 0.0
                             || material_4_child_1_child_1_reflective[1] > 0.0
                             || material_4_child_1_child_1_reflective[2] > 0.0;

    material_4_child_1_child_1->Tr = 0.9000000000;
    material_4_child_1_child_1->Ns = 200.0000000000;
    material_4_child_1_child_1->Ni = 1.0000000000;
    material_4_child_1_child_1->casts_shadow = false;
    material_set_pattern(material_4_child_1_child_1, map_Ka, pattern_4_child_1_child_1_Ka);
    material_set_pattern(material_4_child_1_child_1, map_Kd, pattern_4_child_1_child_1_Kd);
    material_set_pattern(material_4_child_1_child_1, map_Ks, pattern_4_child_1_child_1_Ks);
    material_set_pattern(material_4_child_1_child_1, map_Ns, pattern_4_child_1_child_1_Ns);
    material_set_pattern(material_4_child_1_child_1, map_d, pattern_4_child_1_child_1_d);
    material_set_pattern(material_4_child_1_child_1, map_bump, pattern_4_child_1_child_1_bump);
    material_set_pattern(material_4_child_1_child_1, map_disp, pattern_4_child_1_child_1_disp);
    material_set_pattern(material_4_child_1_child_1, map_refl, pattern_4_child_1_child_1_refl);

    Matrix transform_4_child_1_child_1, transform_4_child_1_child_1_tmp;
    matrix_identity(transform_4_child_1_child_1);
    matrix_translate(1.0000000000, 1.0000000000, 1.0000000000, transform_4_child_1_child_1_tmp);
    transform_chain(transform_4_child_1_child_1_tmp, transform_4_child_1_child_1);
    matrix_scale(3.7333500000, 2.5845000000, 1.6283000000, transform_4_child_1_child_1_tmp);
    transform_chain(transform_4_child_1_child_1_tmp, transform_4_child_1_child_1);
    matrix_translate(-3.9863000000, -0.1217000000, -1.1820000000, transform_4_child_1_child_1_tmp);
    transform_chain(transform_4_child_1_child_1_tmp, transform_4_child_1_child_1);
    matrix_translate(0.0000000000, 0.1216900000, 0.0000000000, transform_4_child_1_child_1_tmp);
    transform_chain(transform_4_child_1_child_1_tmp, transform_4_child_1_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_4_child_1_child_1_tmp);
    transform_chain(transform_4_child_1_child_1_tmp, transform_4_child_1_child_1);

    Shape shape_4_child_1_child_1 = shape_4_child_1_children + 1;
    cube(shape_4_child_1_child_1);
    shape_set_material(shape_4_child_1_child_1, material_4_child_1_child_1);
    shape_set_transform(shape_4_child_1_child_1, transform_4_child_1_child_1);

    /* end children for 4_child_1 */

    Matrix transform_4_child_1, transform_4_child_1_tmp;
    matrix_identity(transform_4_child_1);
    matrix_rotate_y(3.3000000000, transform_4_child_1_tmp);
    transform_chain(transform_4_child_1_tmp, transform_4_child_1);
    matrix_scale(0.5000000000, 0.5000000000, 0.5000000000, transform_4_child_1_tmp);
    transform_chain(transform_4_child_1_tmp, transform_4_child_1);

    Shape shape_4_child_1 = shape_4_children + 1;
    group(shape_4_child_1, shape_4_child_1_children, 2);
    //shape_free(shape_4_child_1_children);
    shape_set_transform(shape_4_child_1, transform_4_child_1);

    /* end children for 4 */

    Matrix transform_4;
    matrix_translate(4.0000000000, 0.0000000000, -2.0000000000, transform_4);
    Shape shape_4 = all_shapes + 4;
    group(shape_4, shape_4_children, 2);
    //shape_free(shape_4_children);
    shape_set_transform(shape_4, transform_4);

    /* end shape 4 */
    /* shape 5 */
    
    /* children for 5 */
    Shape shape_5_children = array_of_shapes(2);

    
        Pattern pattern_5_child_0_Ka = NULL;
    Pattern pattern_5_child_0_Kd = NULL;
    Pattern pattern_5_child_0_Ks = NULL;
    Pattern pattern_5_child_0_Ns = NULL;
    Pattern pattern_5_child_0_bump = NULL;
    Pattern pattern_5_child_0_disp = NULL;
    Pattern pattern_5_child_0_refl = NULL;
    Pattern pattern_5_child_0_d = NULL;
    Color material_5_child_0_color_raw = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_5_child_0_reflective = color(0.2000000000, 0.2000000000, 0.2000000000);
    Color material_5_child_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5_child_0 = material_alloc();
    color_space_fn(material_5_child_0_color_raw, material_5_child_0->Ka);
    color_space_fn(material_5_child_0_color_raw, material_5_child_0->Kd);
    color_space_fn(material_5_child_0_color_raw, material_5_child_0->Ks);
    color_scale(material_5_child_0->Ka, 0.0000000000);
    color_scale(material_5_child_0->Kd, 0.8000000000);
    color_scale(material_5_child_0->Ks, 0.0000000000);
    rgb_to_rgb(material_5_child_0_reflective, material_5_child_0->refl);
    rgb_to_rgb(material_5_child_0_refractive, material_5_child_0->Tf);
    material_5_child_0->reflective = material_5_child_0_reflective[0] > 0.0
                             || material_5_child_0_reflective[1] > 0.0
                             || material_5_child_0_reflective[2] > 0.0;

    material_5_child_0->Tr = 0.0000000000;
    material_5_child_0->Ns = 200.0000000000;
    material_5_child_0->Ni = 1.0000000000;
    material_5_child_0->casts_shadow = true;
    material_set_pattern(material_5_child_0, map_Ka, pattern_5_child_0_Ka);
    material_set_pattern(material_5_child_0, map_Kd, pattern_5_child_0_Kd);
    material_set_pattern(material_5_child_0, map_Ks, pattern_5_child_0_Ks);
    material_set_pattern(material_5_child_0, map_Ns, pattern_5_child_0_Ns);
    material_set_pattern(material_5_child_0, map_d, pattern_5_child_0_d);
    material_set_pattern(material_5_child_0, map_bump, pattern_5_child_0_bump);
    material_set_pattern(material_5_child_0, map_disp, pattern_5_child_0_disp);
    material_set_pattern(material_5_child_0, map_refl, pattern_5_child_0_refl);

    Matrix transform_5_child_0;
    matrix_identity(transform_5_child_0);
    Shape shape_5_child_0 = shape_5_children + 0;
    cylinder(shape_5_child_0);
    shape_set_material(shape_5_child_0, material_5_child_0);
    shape_set_transform(shape_5_child_0, transform_5_child_0);
    shape_5_child_0->fields.cylinder.minimum = -0.1500000000;
    shape_5_child_0->fields.cylinder.maximum = 0.0000000000;
    shape_5_child_0->fields.cylinder.closed = true;


        Pattern pattern_5_child_1_Ka = NULL;
    Pattern pattern_5_child_1_Kd = NULL;
    Pattern pattern_5_child_1_Ks = NULL;
    Pattern pattern_5_child_1_Ns = NULL;
    Pattern pattern_5_child_1_bump = NULL;
    Pattern pattern_5_child_1_disp = NULL;
    Pattern pattern_5_child_1_refl = NULL;
    Pattern pattern_5_child_1_d = NULL;
    Color material_5_child_1_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_5_child_1_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_5_child_1_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_5_child_1 = material_alloc();
    color_space_fn(material_5_child_1_color_raw, material_5_child_1->Ka);
    color_space_fn(material_5_child_1_color_raw, material_5_child_1->Kd);
    color_space_fn(material_5_child_1_color_raw, material_5_child_1->Ks);
    color_scale(material_5_child_1->Ka, 0.1000000000);
    color_scale(material_5_child_1->Kd, 0.6000000000);
    color_scale(material_5_child_1->Ks, 0.8000000000);
    rgb_to_rgb(material_5_child_1_reflective, material_5_child_1->refl);
    rgb_to_rgb(material_5_child_1_refractive, material_5_child_1->Tf);
    material_5_child_1->reflective = material_5_child_1_reflective[0] > 0.0
                             || material_5_child_1_reflective[1] > 0.0
                             || material_5_child_1_reflective[2] > 0.0;

    material_5_child_1->Tr = 0.0000000000;
    material_5_child_1->Ns = 15.0000000000;
    material_5_child_1->Ni = 1.0000000000;
    material_5_child_1->casts_shadow = true;
    material_set_pattern(material_5_child_1, map_Ka, pattern_5_child_1_Ka);
    material_set_pattern(material_5_child_1, map_Kd, pattern_5_child_1_Kd);
    material_set_pattern(material_5_child_1, map_Ks, pattern_5_child_1_Ks);
    material_set_pattern(material_5_child_1, map_Ns, pattern_5_child_1_Ns);
    material_set_pattern(material_5_child_1, map_d, pattern_5_child_1_d);
    material_set_pattern(material_5_child_1, map_bump, pattern_5_child_1_bump);
    material_set_pattern(material_5_child_1, map_disp, pattern_5_child_1_disp);
    material_set_pattern(material_5_child_1, map_refl, pattern_5_child_1_refl);

    Matrix transform_5_child_1, transform_5_child_1_tmp;
    matrix_identity(transform_5_child_1);
    matrix_translate(0.0000000000, 0.1217000000, 0.0000000000, transform_5_child_1_tmp);
    transform_chain(transform_5_child_1_tmp, transform_5_child_1);
    matrix_scale(0.2680000000, 0.2680000000, 0.2680000000, transform_5_child_1_tmp);
    transform_chain(transform_5_child_1_tmp, transform_5_child_1);
    matrix_rotate_y(3.1415000000, transform_5_child_1_tmp);
    transform_chain(transform_5_child_1_tmp, transform_5_child_1);

    Shape shape_5_child_1 = shape_5_children + 1;
    shape_copy(shape_4_child_1_child_0, NULL, shape_5_child_1);
    shape_set_material_recursive(shape_5_child_1, material_5_child_1);
    shape_set_transform(shape_5_child_1, transform_5_child_1);

    /* end children for 5 */

    Matrix transform_5;
    matrix_translate(0.0000000000, 0.5000000000, -4.0000000000, transform_5);
    Shape shape_5 = all_shapes + 5;
    group(shape_5, shape_5_children, 2);
    //shape_free(shape_5_children);
    shape_set_transform(shape_5, transform_5);

    /* end shape 5 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 6);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 4;
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

